# GPU tests then bench variants; stops on anything but a clean pass or plain test failures.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gputest.log 2>&1
rc=$?
tail -5 gpurun_out/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/variants.sh
