for f in gpurun_out/v_*.log; do python -c "
import json,sys
ls=[x for x in open('$f') if x.startswith('{')]
if not ls: print('$f', 'NO RESULT'); sys.exit()
d=json.loads(ls[-1])
print('%-28s %8.2f G/s %9.3f ms %8.1f GB/s reruns=%s' % ('$f', d['value']/1e9, d['ms_per_step'], d['roofline']['achieved'], d['tier_reruns']))"; done
