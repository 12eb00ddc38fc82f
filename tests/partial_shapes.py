"""Partial-replication shapes (shard_count > 1, graph/mod.rs:82-406) driven
the same way on the CPU oracle and on the GPU executor handle.

The reference has no unit test of the executor with shard_count > 1 (its
partial-replication tests run Tempo / Atlas in run mode over TCP,
fantoch_ps/src/protocol/mod.rs:278-333), so these shapes are parity vs the
restatement (oracle/graph_oracle.hpp): a hand-derived known answer from the
code of tarjan.rs:148-166 / mod.rs:394-402 / index.rs:168-202, and seeded
random scenarios in which the driver answers every out-request with
RequestReply::Info or ::Executed after a delay, as the shard owning the dot
would."""
import numpy as np

# n = 2 processes per shard, 2 shards: ids 1, 2 (shard 0) and 3, 4 (shard 1);
# the executor under test is process 1 of shard 0.
KAT = dict(
    n=2, shards=2, shard=0,
    script=[
        # A = (1,1) depends on B = (3,1), replicated by shard 1 only: missing,
        # not mine -> requested from shard 1
        ("add", (1, 1), [((3, 1), 0b10)]),
        # C = (2,1) depends on B (already a PendingIndex key: no new request)
        # and D = (4,1), replicated by both shards (mine: no request); the first
        # search collects both, C waits on both
        ("add", (2, 1), [((3, 1), 0b10), ((4, 1), 0b11)]),
        # RequestReply::Executed{B}: A executes; C is retried and still misses D
        ("executed", (3, 1)),
        # D arrives: D, then C execute
        ("add", (4, 1), []),
    ],
    expect=[
        dict(executed=[], requests=[(1, (3, 1))], to_executors=[]),
        dict(executed=[], requests=[], to_executors=[]),
        dict(executed=[(1, 1)], requests=[], to_executors=[(1, 1), (3, 1)]),
        dict(executed=[(4, 1), (2, 1)], requests=[], to_executors=[(2, 1), (4, 1)]),
    ],
)


def scenario(seed, n=2, shards=2, shard=0, cmds=240, window=10, fwd_pct=20, both_pct=40, reply_delay=6):
    """A seeded global command history and the script one shard-`shard`
    executor sees: Adds of the commands its shard replicates (window-shuffled),
    and the replies to its requests, produced by `drive`."""
    rng = np.random.default_rng(seed)
    seqs = {}
    hist = []  # (dot, mask, [dep indices])
    for i in range(cmds):
        home = int(rng.integers(shards))
        src = 1 + home * n + int(rng.integers(n))
        seqs[src] = seqs.get(src, 0) + 1
        mask = (1 << shards) - 1 if rng.integers(100) < both_pct else 1 << home
        deps = set()
        for _ in range(int(rng.integers(0, 4))):
            if i:
                deps.add(int(rng.integers(max(0, i - window), i)))
        if rng.integers(100) < fwd_pct and i + 1 < cmds:
            deps.add(int(rng.integers(i + 1, min(cmds, i + window))))
        hist.append(((src, seqs[src]), mask, sorted(deps)))
    mine = [i for i, (_, m, _) in enumerate(hist) if (m >> shard) & 1]
    order = []
    buf = list(mine)
    while buf:  # window shuffle: deliver one of the first `window` remaining
        j = int(rng.integers(min(window, len(buf))))
        order.append(buf.pop(j))
    return hist, order


def drive(hist, order, backend, reply_delay=6, seed=0):
    """Runs the script on `backend` (an object with add(dot, deps, masks, t),
    executed(dots, t), pull() -> (executed dots, requests, to_executors)) and
    returns the per-step observations.  Requests are answered reply_delay
    steps later with Info (the command) or Executed, chosen by the dot."""
    by_dot = {d: (d, m, deps) for d, m, deps in hist}
    idx_dot = [d for d, _, _ in hist]
    replies = []  # (due, dot)
    log = []
    t = 0

    def add_cmd(dot):
        # an own command and an Info reply (a command of other shards) both
        # carry the command's shard set (Command::shards)
        _, m, deps = by_dot[dot]
        backend.add(dot, [idx_dot[k] for k in deps], [hist[k][1] for k in deps], t, cmd_shards=m)

    def step():
        log.append(backend.pull())
        for _shard, dot in log[-1][1]:
            replies.append((t + reply_delay, dot))

    for i in order:
        t += 1
        add_cmd(idx_dot[i])
        step()
        due = [r for r in replies if r[0] <= t]
        replies[:] = [r for r in replies if r[0] > t]
        for _, dot in sorted(due):
            t += 1
            if (hash((dot, seed)) & 1) == 0:
                add_cmd(dot)  # RequestReply::Info
            else:
                backend.executed([dot], t)  # RequestReply::Executed
            step()
    while replies:
        due = sorted(replies)
        replies.clear()
        for _, dot in due:
            t += 1
            if (hash((dot, seed)) & 1) == 0:
                add_cmd(dot)
            else:
                backend.executed([dot], t)
            step()
    return log


class OracleBackend:
    def __init__(self, n, shards, shard):
        from oracle import oracle_lib
        self.g = oracle_lib.Graph(1 + shard * n, n, shard_id=shard, shard_count=shards)

    def add(self, dot, deps, masks, t, cmd_shards=0):
        self.g.handle_add_sharded(dot, deps, masks, t)

    def executed(self, dots, t):
        for d in dots:
            self.g.executed_reply(d, t)

    def pull(self):
        return ([d for d, _, _ in self.g.drain()], self.g.requests(), self.g.to_executors())

    def waits(self):
        return self.g.waits()


class GpuBackend:
    def __init__(self, n, shards, shard):
        from fantoch_amd.executor import GraphExecutor
        self.ex = GraphExecutor(1 + shard * n, shard, n, shard_count=shards, monitor=False)

    def add(self, dot, deps, masks, t, cmd_shards=0):
        self.ex.handle_add_sharded(dot, dot, [0], deps, masks, t, cmd_shards=cmd_shards)

    def executed(self, dots, t):
        self.ex.handle_executed(dots, t)

    def pull(self):
        return ([d for d, _ in self.ex.drain_dots()], self.ex.requests(), self.ex.to_executors())

    def waits(self):
        return sorted((d, w) for d, w in self.ex.pending() if w != (0, 0))


def run_kat(backend):
    out = []
    t = 0
    for op in KAT["script"]:
        t += 1
        if op[0] == "add":
            backend.add(op[1], [d for d, _ in op[2]], [m for _, m in op[2]], t)
        else:
            backend.executed([op[1]], t)
        out.append(backend.pull())
    return out


def drive_serving(hist, order, backend, seed=0, req_pct=30):
    """The main executor of shard 0 takes the Adds of its commands; its clone
    (executor index 1) gets every step's executed dots (to_executors ->
    GraphExecutionInfo::Executed) and Requests from shard 1 for random dots of
    shard-0 commands (delivered, pending or not yet added), with a cleanup
    every third step.  Returns the replies per step."""
    rng = np.random.default_rng(seed)
    by_dot = {d: (m, deps) for d, m, deps in hist}
    idx_dot = [d for d, _, _ in hist]
    mine = [idx_dot[i] for i in order]
    log = []
    for t, i in enumerate(order):
        d = idx_dot[i]
        m, deps = by_dot[d]
        backend.add(d, [idx_dot[k] for k in deps], [hist[k][1] for k in deps], t)
        backend.clone_executed(backend.pull()[2])
        if rng.integers(100) < req_pct:
            k = int(rng.integers(1, 4))
            backend.request(1, [mine[int(j)] for j in rng.integers(0, len(mine), size=k)])
        if t % 3 == 2:
            backend.cleanup()
        log.append(backend.replies())
    backend.cleanup()
    log.append(backend.replies())
    return log


class OracleServing(OracleBackend):
    def __init__(self, n, shards, shard):
        super().__init__(n, shards, shard)
        self.c = self.g.clone()

    def clone_executed(self, dots):
        self.c.handle_executed(dots)

    def request(self, from_shard, dots):
        self.c.handle_request(from_shard, dots)

    def cleanup(self):
        self.c.cleanup()

    def replies(self):
        return [(to, kind, dot, deps) for to, kind, dot, deps in self.c.replies()]


class GpuServing(GpuBackend):
    def __init__(self, n, shards, shard):
        super().__init__(n, shards, shard)
        self.c = self.ex.clone()

    def clone_executed(self, dots):
        self.c.handle_executed(dots)

    def request(self, from_shard, dots):
        self.c.handle_request(from_shard, dots)

    def cleanup(self):
        self.c.cleanup()

    def replies(self):
        return self.c.replies()
