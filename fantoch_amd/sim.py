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
         instance=0):
    """One instance (Config + Workload + placement), regions as planet indices.
    Defaults are fantoch_ps/src/bin/simulation.rs's (config! macro: GC and
    executed notifications every 10 ms; pool 1, 1 key per command, run(None))."""
    s = _lib.SimSpec()
    s.seed, s.instance, s.protocol, s.n, s.f = seed, instance, protocol, n, f
    s.gc_interval_ms, s.executed_notification_ms = gc_interval_ms, executed_notification_ms
    s.clients_per_region, s.commands_per_client = clients_per_region, commands_per_client
    s.keys_per_command, s.conflict_rate, s.pool_size = keys_per_command, conflict_rate, pool_size
    s.read_only_pct, s.extra_sim_time_ms, s.reorder_messages, s.nfr = 0, extra_sim_time_ms, 0, 0
    s.num_client_regions = len(client_regions)
    for i, r in enumerate(process_regions):
        s.process_regions[i] = r
    for i, r in enumerate(client_regions):
        s.client_regions[i] = r
    return s


class Result:
    """Host copies of one batch's outputs."""

    def __init__(self, specs, executed, executed_len, latency_log, latency_hist, chain, delay,
                 stats, err, exec_cap, lat_cap):
        self.specs = specs
        self.n = specs[0].n
        self.C = specs[0].clients_per_region * specs[0].num_client_regions
        self.executed_len = executed_len.reshape(len(specs), self.n)
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

    def trace(self, i):
        return int(self.stats[i, _lib.FX_SIM_STAT_TRACE])

    def events(self, i):
        return int(self.stats[i, _lib.FX_SIM_STAT_EVENTS])

    def end_ms(self, i):
        return int(self.stats[i, _lib.FX_SIM_STAT_END_MS])


def run(specs, planet=None, exec_cap=None, lat_cap=None, lat_bins=8192, chain_bins=256,
        delay_bins=8192, ring_entries=0, dot_slots=0, max_events=0, flags=0, stream=None):
    """Simulates every instance of `specs` on the GPU; returns a Result."""
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
    host = (_lib.SimSpec * N)(*specs)
    dspec = DeviceBuffer(ctypes.sizeof(host))
    check(lib.fx_dev_h2d(dspec.ptr, ctypes.addressof(host), ctypes.sizeof(host), stream), "h2d")
    ping, rank = planet.device()
    out = {}
    sizes = {"executed": N * s0.n * exec_cap * 4, "executed_len": N * s0.n * 4,
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
                       lat_bins, chain_bins, delay_bins, 0)
    reruns = ctypes.c_uint32()
    check(lib.fx_sim_run_tiered(ctypes.byref(b), ctypes.byref(o), stream, ctypes.byref(reruns)),
          "fx_sim_run_tiered")
    check(lib.fx_dev_synchronize(stream), "fx_sim_run sync")
    d = lambda k, dt, cnt: out[k].download(dt, cnt, stream)
    res = Result(specs, d("executed", np.uint32, N * s0.n * exec_cap),
                 d("executed_len", np.uint32, N * s0.n),
                 d("latency_log", np.uint32, N * C * lat_cap) if lat_cap else None,
                 d("latency_hist", np.uint64, planet.R * lat_bins).reshape(planet.R, lat_bins),
                 d("chain", np.uint64, chain_bins), d("delay", np.uint64, delay_bins),
                 d("stats", np.uint64, N * _lib.FX_SIM_STATS), d("err", np.uint32, N),
                 exec_cap, lat_cap)
    res.reruns = int(reruns.value)  # instances rerun with larger tables (fx_sim_run_tiered)
    return res
