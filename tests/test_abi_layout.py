"""The ctypes mirrors in fantoch_amd/_lib.py against the C-ABI header
(include/fantoch_amd.h): every struct's size and every field's offset, as
gcc lays them out.  CPU only (no library call): a binding whose layout drifts
from the header (a field added at the end, as fx_cut_stats.single_segments in
round 6) fails here instead of corrupting memory on the GPU box."""
import ctypes
import os
import shutil
import subprocess
import tempfile

import pytest

from fantoch_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# ctypes mirror -> C typedef
PAIRS = {
    "StreamBatch": "fx_stream_batch",
    "OrderBatch": "fx_order_batch",
    "PredBatch": "fx_pred_batch",
    "CutStats": "fx_cut_stats",
    "HistBatch": "fx_hist_batch",
    "TierInfo": "fx_tier_info",
    "SynthParams": "fx_synth_params",
    "Config": "fx_config",
    "CDot": "fx_dot",
    "CRifl": "fx_rifl",
    "ExecutorResultC": "fx_executor_result",
    "RequestReplyC": "fx_request_reply",
    "LogSummary": "fx_log_summary",
    "LogAdd": "fx_log_add",
    "HistStats": "fx_hist_stats",
    "SimSpec": "fx_sim_spec",
    "SimBatch": "fx_sim_batch",
    "SimOutput": "fx_sim_output",
}


def _c_layout():
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "fantoch_amd.h"', "int main(void) {"]
    for py, c in PAIRS.items():
        lines.append('  printf("%s size %%zu\\n", sizeof(%s));' % (py, c))
        for name, _ in getattr(_lib, py)._fields_:
            lines.append('  printf("%s %s %%zu\\n", offsetof(%s, %s));' % (py, name, c, name))
    lines += ["  return 0;", "}"]
    d = tempfile.mkdtemp()
    try:
        src, exe = os.path.join(d, "abi.c"), os.path.join(d, "abi")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", exe, src], check=True,
                       capture_output=True, text=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(d, ignore_errors=True)
    layout = {}
    for ln in out.split("\n"):
        if ln:
            a, b, v = ln.split()
            layout[(a, b)] = int(v)
    return layout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_ctypes_mirrors_match_the_header():
    layout = _c_layout()
    for py in PAIRS:
        cls = getattr(_lib, py)
        assert ctypes.sizeof(cls) == layout[(py, "size")], py
        for name, _ in cls._fields_:
            assert getattr(cls, name).offset == layout[(py, name)], (py, name)
