"""PMC figures of the bench modes' dominant kernels, for the roofline blocks.

rocprofv3 counter passes of one bench mode (tools/mode_pmc.sh) are summarised
by tools/mode_pmc_summary.py into profiles/pmc_<mode>.json: the workload key
(the bench arguments that shape the work), the dominant kernel, its HBM
traffic per launch (FETCH_SIZE + WRITE_SIZE, each in its own pass) and its
issue figures (SQ_INSTS_* and wave counters against GRBM_GUI_ACTIVE).  A bench
line takes them when its own workload key matches, so a number never describes
another workload.  Conventions (MI355X_MICROARCH.md, HBM / rocprofv3 section):
FETCH_SIZE and WRITE_SIZE are KB; FETCH_SIZE is reported raw and x2 (the gfx950
correction for wide coalesced reads; tools/fetch_calib.hip measured 0.5x the
bytes of a coalesced read at both 4 B and 16 B per lane on this box, so x2 is
the one used for `traffic`); GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles."""
import json
import os

ROOT = os.path.dirname(os.path.abspath(__file__))
# bench arguments that do not change the work of a launch
_NOT_WORK = {"gpus", "steps", "warmup", "cpu_baseline_seconds", "no_cpu_baseline", "traffic_json", "pmc_key"}


# arguments that shape only --mode huge's stream
_HUGE_ONLY = {"huge_shape", "key_pool", "horizon"}


def workload_key(args):
    skip = _NOT_WORK | (set() if getattr(args, "mode", None) == "huge" else _HUGE_ONLY)
    return json.dumps({k: v for k, v in sorted(vars(args).items()) if k not in skip}, sort_keys=True)


def path(mode):
    return os.path.join(ROOT, "profiles", "pmc_%s.json" % mode)


def load(mode, args):
    """The PMC summary of this mode if it was measured on this workload, else None."""
    p = path(mode)
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
    except Exception:
        return None
    key = getattr(args, "pmc_key", None) or workload_key(args)
    return d if d.get("workload_key") == key else None


def attach(roof, pm, alg_bytes_per_launch):
    """roofline.traffic (HBM bytes per launch of the dominant kernel, from the
    counters), its ratio to the §8(d) algorithmic bytes, and roofline.issue."""
    if not pm:
        roof.setdefault("traffic", None)
        return roof
    t = pm.get("hbm_bytes_per_launch")
    roof["traffic"] = t
    if t and alg_bytes_per_launch:
        roof["traffic_over_alg"] = round(t / alg_bytes_per_launch, 4)
    for k in ("read_bytes_x2", "read_bytes_raw", "write_bytes"):
        if k in pm:
            roof["traffic_" + k] = pm[k]
    if pm.get("issue"):
        roof["issue"] = dict(pm["issue"], source="profiles/pmc_%s.json (%s)" % (pm.get("mode"), pm.get("source")))
    # north_star's rocprof figures beside achieved GB/s: LDS bank conflicts
    # (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) and wave occupancy
    # (SQ_WAVE_CYCLES per CU cycle), from the same counter record
    if pm.get("lds_bank_conflict_frac") is not None:
        roof["lds_bank_conflict_frac"] = pm["lds_bank_conflict_frac"]
    if (pm.get("issue") or {}).get("mean_waves_per_cu") is not None:
        roof["mean_waves_per_cu"] = pm["issue"]["mean_waves_per_cu"]
    if pm.get("kernel_pattern"):
        roof["pmc_kernel"] = pm["kernel_pattern"]
    return roof
