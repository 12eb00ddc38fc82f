"""Where the Basic runner-KAT instance stops on the all-on-chip kernel (one
fx_sim_run, no capacity reruns): error and source line of the first failure."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fantoch_amd import _lib  # noqa: E402
from fantoch_amd import sim as S  # noqa: E402

pl = S.Planet()
for f in (0, 1):
    for cpp in (1, 10):
        s = S.spec(S.BASIC, 3, f, pl.ids(["asia-east1", "us-central1", "us-west1"]), pl.ids(["us-west1", "us-west2"]),
                   clients_per_region=cpp, commands_per_client=1000, conflict_rate=100, pool_size=1,
                   gc_interval_ms=100, executed_notification_ms=50, extra_sim_time_ms=1000)
        for dots in (0, 256):
            r = S.run([s], pl, tiered=False, dot_slots=dots)
            print("f", f, "cpp", cpp, "dots", dots, "err", int(r.err[0]), "site",
                  int(r.stats[0, _lib.FX_SIM_STAT_ERR_SITE]), "events", r.events(0), "end", r.end_ms(0),
                  "exec", [len(e) for e in r.executed(0)], "stable", list(r.stable(0)), flush=True)
