"""Batched simulator on the GPU (fx_sim_run): one wavefront per simulated instance.

The reference's entry point is `Runner::new(planet, config, workload,
clients_per_process, process_regions, client_regions)` + `Runner::run`
(fantoch/src/sim/runner.rs:64-231), driven over many (protocol config, seed,
conflict rate, region placement) tuples by `fantoch_ps/src/bin/simulation.rs`.
Here a `Spec` is one such instance and `run(specs)` simulates a whole batch in
one launch; results come back per instance (per-process execution order,
per-command client latencies, protocol counters) plus batch histograms.
Regions are planet indices in name order (canonical C12, see `Planet`).
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check
from .device import DeviceBuffer

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "latency_gcp")
ATLAS, EPAXOS, BASIC = _lib.FX_PROTOCOL_ATLAS, _lib.FX_PROTOCOL_EPAXOS, _lib.FX_PROTOCOL_BASIC
# regions of simulation.rs:148-158 (gcp_planet), in the order the binary lists them
GCP5 = ["asia-south1", "europe-north1", "southamerica-east1", "australia-southeast1", "europe-west1"]


class Planet:
    """Planet::from(dir) (planet/mod.rs:38-54) through fx_planet_load."""

    STRIDE = 32

    def __init__(self, data_dir=DATA_DIR):
        lib = _lib.load()
        R = ctypes.c_uint32()
        self.ping = np.zeros((self.STRIDE, self.STRIDE), np.uint16)
        self.rank = np.zeros((self.STRIDE, self.STRIDE), np.uint8)
        names = ctypes.create_string_buffer(4096)
        check(lib.fx_planet_load(data_dir.encode(), self.STRIDE, ctypes.byref(R), names, 4096,
                                 self.ping.ctypes.data, self.rank.ctypes.data), "fx_planet_load")
        self.regions = names.value.decode().split()
        self.R = R.value
        self.index = {r: i for i, r in enumerate(self.regions)}
        self._dev = None

    def device(self):
        if self._dev is None:
            dp = DeviceBuffer(self.ping.nbytes)
            dp.upload(self.ping)
            dr = DeviceBuffer(self.rank.nbytes)
            dr.upload(self.rank)
            self._dev = (dp, dr)
        return self._dev

    def ids(self, names):
        return [self.index[r] for r in names]


def spec(protocol, n, f, process_regions, client_regions, clients_per_region=1,
         commands_per_client=1000, keys_per_command=1, conflict_rate=2, pool_size=1,
         gc_interval_ms=10, executed_notification_ms=10, extra_sim_time_ms=-1, seed=0,
         instance=0, read_only_pct=0, reorder=False, nfr=False):
    """One instance (Config + Workload + placement), regions as planet indices.
    Defaults are fantoch_ps/src/bin/simulation.rs's (config! macro: GC and
    executed notifications every 10 ms; pool 1, 1 key per command, run(None)).
    read_only_pct = Workload::set_read_only_percentage, reorder =
    Runner::reorder_messages, nfr = Config::set_nfr."""
    s = _lib.SimSpec()
    s.seed, s.instance, s.protocol, s.n, s.f = seed, instance, protocol, n, f
    s.gc_interval_ms, s.executed_notification_ms = gc_interval_ms, executed_notification_ms
    s.clients_per_region, s.commands_per_client = clients_per_region, commands_per_client
    s.keys_per_command, s.conflict_rate, s.pool_size = keys_per_command, conflict_rate, pool_size
    s.read_only_pct, s.extra_sim_time_ms = read_only_pct, extra_sim_time_ms
    s.reorder_messages, s.nfr = int(bool(reorder)), int(bool(nfr))
    s.num_client_regions = len(client_regions)
    for i, r in enumerate(process_regions):
        s.process_regions[i] = r
    for i, r in enumerate(client_regions):
        s.client_regions[i] = r
    return s


# ------------------------------------------------------------- workload
# The kernels' workload (Workload::gen_cmd, workload.rs:142-197, with the
# canonical C6 counter RNG) restated on the host, so a run's commands can be
# named without the device: the keys and read-only flag of command idx
# (0-based) of client cid (1-based).
_M64 = (1 << 64) - 1


def _mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def _sim_rand(seed, inst, client, idx, purpose):
    x = _mix64(seed ^ 0x5851F42D4C957F2D)
    x = _mix64((x + inst) & _M64)
    x = _mix64((x + client) & _M64)
    return _mix64((x + (((idx << 8) | purpose) & _M64)) & _M64)


def command(s, cid, idx):
    """(keys ascending, read_only) of command idx of client cid (1-based)."""
    keys, draw = [], 0
    while len(keys) < s.keys_per_command:
        if s.conflict_rate == 0:
            conflict = False
        elif s.conflict_rate >= 100:
            conflict = True
        else:
            conflict = _sim_rand(s.seed, s.instance, cid, idx * 64 + draw, 1) % 100 < s.conflict_rate
        if conflict:
            key = 0 if s.pool_size <= 1 else _sim_rand(s.seed, s.instance, cid, idx * 64 + draw, 2) % s.pool_size
        else:
            key = s.pool_size + cid
        draw += 1
        if key not in keys:
            keys.append(key)
    if s.read_only_pct == 0:
        ro = False
    elif s.read_only_pct >= 100:
        ro = True
    else:
        ro = _sim_rand(s.seed, s.instance, cid, idx, 3) % 100 < s.read_only_pct
    return sorted(keys), ro


class Result:
    """Host copies of one batch's outputs."""

    def __init__(self, specs, executed, executed_len, latency_log, latency_hist, chain, delay,
                 stats, err, exec_cap, lat_cap, dot_client=None):
        self.specs = specs
        self.n = specs[0].n
        self.C = specs[0].clients_per_region * specs[0].num_client_regions
        self.exec_cap = exec_cap
        self.executed_len = executed_len.reshape(len(specs), self.n)
        self._dot_client = dot_client.reshape(len(specs), self.n, exec_cap) if dot_client is not None else None
        self._executed = executed.reshape(len(specs), self.n, exec_cap) if executed is not None else None
        self._lat = latency_log.reshape(len(specs), self.C, lat_cap) if latency_log is not None else None
        self.latency_hist = latency_hist
        self.chain = chain
        self.delay = delay
        self.stats = stats.reshape(len(specs), _lib.FX_SIM_STATS)
        self.err = err

    def executed(self, i):
        """Per-process execution order of instance i: list of packed-dot arrays."""
        return [self._executed[i, p, :int(self.executed_len[i, p])].copy() for p in range(self.n)]

    def latencies(self, i):
        """[C][commands] client latencies (ms) of instance i, client id order."""
        return self._lat[i]

    def fast(self, i):
        return self.stats[i, _lib.FX_SIM_STAT_FAST:_lib.FX_SIM_STAT_FAST + self.n]

    def slow(self, i):
        return self.stats[i, _lib.FX_SIM_STAT_SLOW:_lib.FX_SIM_STAT_SLOW + self.n]

    def stable(self, i):
        return self.stats[i, _lib.FX_SIM_STAT_STABLE:_lib.FX_SIM_STAT_STABLE + self.n]

    def fast_reads(self, i):
        return self.stats[i, _lib.FX_SIM_STAT_FAST_READS:_lib.FX_SIM_STAT_FAST_READS + self.n]

    def slow_reads(self, i):
        return self.stats[i, _lib.FX_SIM_STAT_SLOW_READS:_lib.FX_SIM_STAT_SLOW_READS + self.n]

    def rifls(self, i):
        """Per process, the rifl (client id, command seq) of every executed
        command of instance i in execution order: dot (p, s) was submitted by
        client dot_client[p][s - 1], and a client's k-th dot is its command k."""
        dc = self._dot_client[i]
        seqno = {}
        for p in range(self.n):
            per = {}
            for s in range(1, self.exec_cap + 1):
                c = int(dc[p, s - 1])
                if c:
                    per[c] = per.get(c, 0) + 1
                    seqno[(p + 1, s)] = (c, per[c])
        out = []
        for order in self.executed(i):
            out.append([seqno[(int(d) >> 24, int(d) & 0xFFFFFF)] for d in order])
        return out

    def monitors(self, i):
        """ExecutionOrderMonitor of every process (executor/monitor.rs:8-55,
        command.rs:147-162): per key, the rifls of the non-read-only commands
        in execution order."""
        s = self.specs[i]
        out = []
        for rifls in self.rifls(i):
            mon = {}
            for c, q in rifls:
                keys, ro = command(s, c, q - 1)
                if ro:
                    continue
                for k in keys:
                    mon.setdefault(k, []).append((c, q))
            out.append(mon)
        return out

    def trace(self, i):
        return int(self.stats[i, _lib.FX_SIM_STAT_TRACE])

    def events(self, i):
        return int(self.stats[i, _lib.FX_SIM_STAT_EVENTS])

    def end_ms(self, i):
        return int(self.stats[i, _lib.FX_SIM_STAT_END_MS])


def run(specs, planet=None, exec_cap=None, lat_cap=None, lat_bins=8192, chain_bins=256,
        delay_bins=8192, ring_entries=0, dot_slots=0, max_events=0, flags=0, stream=None,
        large=False, generic=False, tiered=True, before_launch=None, arena_fill=False):
    """Simulates every instance of `specs` on the GPU; returns a Result.
    large=True forces the large-instance kernel (FX_SIM_FLAG_LARGE);
    generic=True the run-time-geometry build of either kernel even for a
    compiled-in geometry (FX_SIM_FLAG_GENERIC); arena_fill=True (tests) the
    large-instance kernel's arena starts filled with 0xA5 bytes instead of
    zeroed (FX_SIM_FLAG_ARENA_FILL); tiered=False: one
    fx_sim_run, instances that outgrow the tables keep FX_ERR_SIM_CAPACITY.
    before_launch(stream): called once the inputs and outputs are on the
    device, right before the launch (diagnostics: tools/sim_poison.py)."""
    lib = _lib.load()
    planet = planet or Planet()
    N = len(specs)
    s0 = specs[0]
    C = s0.clients_per_region * s0.num_client_regions
    cmds = max(s.commands_per_client for s in specs)
    if exec_cap is None:
        exec_cap = C * cmds + 8
    if lat_cap is None:
        lat_cap = cmds
    if not max_events:  # a bound every instance reaches: a stuck run ends with FX_ERR_SIM_EVENTS
        max_events = min(0xFFFFFFFF, 4000 * C * cmds + 10_000_000)
    if large:
        flags |= _lib.FX_SIM_FLAG_LARGE
    if generic:
        flags |= _lib.FX_SIM_FLAG_GENERIC
    if arena_fill:
        flags |= _lib.FX_SIM_FLAG_ARENA_FILL
    host = (_lib.SimSpec * N)(*specs)
    dspec = DeviceBuffer(ctypes.sizeof(host))
    check(lib.fx_dev_h2d(dspec.ptr, ctypes.addressof(host), ctypes.sizeof(host), stream), "h2d")
    ping, rank = planet.device()
    out = {}
    sizes = {"executed": N * s0.n * exec_cap * 4, "executed_len": N * s0.n * 4,
             "dot_client": N * s0.n * exec_cap * 4,
             "latency_log": N * C * max(lat_cap, 1) * 4, "latency_hist": planet.R * lat_bins * 8,
             "chain": chain_bins * 8, "delay": delay_bins * 8, "stats": N * _lib.FX_SIM_STATS * 8,
             "err": N * 4}
    for k, v in sizes.items():
        out[k] = DeviceBuffer(v)
        out[k].zero(stream)
    b = _lib.SimBatch(dspec.ptr, ctypes.addressof(host), N, flags, ping.ptr, rank.ptr, planet.R,
                      Planet.STRIDE, exec_cap, lat_cap, max_events, ring_entries, dot_slots, 0)
    o = _lib.SimOutput(out["executed"].ptr, out["executed_len"].ptr,
                       out["latency_log"].ptr if lat_cap else None, out["latency_hist"].ptr,
                       out["chain"].ptr, out["delay"].ptr, out["stats"].ptr, out["err"].ptr,
                       lat_bins, chain_bins, delay_bins, 0, out["dot_client"].ptr)
    reruns = ctypes.c_uint32()
    if before_launch is not None:
        before_launch(stream)
    if tiered:
        check(lib.fx_sim_run_tiered(ctypes.byref(b), ctypes.byref(o), stream, ctypes.byref(reruns)),
              "fx_sim_run_tiered")
    else:
        check(lib.fx_sim_run(ctypes.byref(b), ctypes.byref(o), stream), "fx_sim_run")
    check(lib.fx_dev_synchronize(stream), "fx_sim_run sync")
    d = lambda k, dt, cnt: out[k].download(dt, cnt, stream)
    res = Result(specs, d("executed", np.uint32, N * s0.n * exec_cap),
                 d("executed_len", np.uint32, N * s0.n),
                 d("latency_log", np.uint32, N * C * lat_cap) if lat_cap else None,
                 d("latency_hist", np.uint64, planet.R * lat_bins).reshape(planet.R, lat_bins),
                 d("chain", np.uint64, chain_bins), d("delay", np.uint64, delay_bins),
                 d("stats", np.uint64, N * _lib.FX_SIM_STATS), d("err", np.uint32, N),
                 exec_cap, lat_cap, d("dot_client", np.uint32, N * s0.n * exec_cap))
    res.reruns = int(reruns.value)  # instances rerun with larger tables (fx_sim_run_tiered)
    return res
