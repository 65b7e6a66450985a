"""Row-sharded clusters: one libswimhip handle per GPU, each owning a contiguous range of observers.

include/swimhip_shard.h is the C ABI. The shards step in lockstep and exchange, per tick, the gossip records and
the SYNC / SYNC_ACK payloads addressed to each other's observers. Two transports:
  * RCCL (production): send/recv groups on the handle's HIP stream over xGMI. The caller only distributes the
    RCCL unique id, e.g. with torch.distributed (rccl_unique_id / ShardedCluster.rccl).
  * HOST: the library stages each exchange through host memory and calls back into Python. GlooExchange runs it
    over a torch.distributed gloo group (one process per rank); ThreadExchange runs W shards inside one process,
    one Python thread per shard (tests on a single GPU).
The readback methods of SimulatedCluster report this shard's observers only; gather_* helpers merge them.
"""
import ctypes as C
import dataclasses
import threading

import numpy as np

from . import _abi
from .cluster import SimulatedCluster, SwimError
from .config import SimConfig


COUNT_MASK = (1 << 48) - 1  # exchange count words: bytes below bit 48, opaque flags above (swimhip_shard.h)


def shard_range(n, world, rank):
    """[lo, hi) observers of a rank: contiguous ranges floor(r N / W) (engine.h shard_lo)."""
    return rank * n // world, (rank + 1) * n // world


def rccl_unique_id(lib):
    buf = (C.c_uint8 * 128)()
    rc = lib.swim_rccl_unique_id(buf)
    if rc != 0:
        raise SwimError(f"swim_rccl_unique_id failed rc={rc}")
    return bytes(buf)


class _HostExchange:
    """Base of the SWIM_TRANSPORT_HOST callbacks: keeps the ctypes thunk alive and reports exceptions."""

    def __init__(self):
        self.error = None
        self.calls = 0

    def _run(self, send, send_bytes, recv, recv_cap, recv_bytes):
        raise NotImplementedError

    def callback(self):
        def cb(ctx, send, sb, recv, cap, rb):
            try:
                self._run(send, sb, recv, cap, rb)
                self.calls += 1
                return 0
            except BaseException as e:  # noqa: BLE001 - reported through swim_step's error code
                self.error = e
                return -1

        self._thunk = _abi.EXCHANGE_FN(cb)
        return self._thunk


class GlooExchange(_HostExchange):
    """All-to-all of per-peer byte blocks over a torch.distributed process group (gloo, CPU tensors)."""

    def __init__(self, group=None):
        super().__init__()
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)

    def _run(self, send, sb, recv, cap, rb):
        import torch
        W = self.world
        words = [int(sb[q]) for q in range(W)]  # bytes in the low 48 bits, flags above (delivered unchanged)
        scounts = [w & COUNT_MASK for w in words]
        sc = torch.tensor(words, dtype=torch.int64)
        rc = torch.empty(W, dtype=torch.int64)
        self.dist.all_to_all_single(rc, sc, group=self.group)
        rwords = [int(x) for x in rc.tolist()]
        rcounts = [w & COUNT_MASK for w in rwords]
        total_s, total_r = sum(scounts), sum(rcounts)
        if total_r > cap:
            raise RuntimeError(f"receive {total_r} bytes > capacity {cap}")
        inp = torch.from_numpy(np.ctypeslib.as_array((C.c_uint8 * max(total_s, 1)).from_address(send)).copy()[:total_s])
        out = torch.empty(total_r, dtype=torch.uint8)
        self.dist.all_to_all_single(out, inp, rcounts, scounts, group=self.group)
        if total_r:
            C.memmove(recv, out.numpy().ctypes.data, total_r)
        for p in range(W):
            rb[p] = rwords[p]


class LoneExchange(_HostExchange):
    """A timing rehearsal of one shard without its peers: every peer "sends" a block of the size this rank sends it,
    all zeros. For slot shards (RUMOR mode) that is a zero gossip-count delta from every other shard, so the shard
    runs its full per-tick work; the results are not the W-shard simulation's (bench.py --rehearse-shard)."""

    def __init__(self, world):
        super().__init__()
        self.world = world

    def _run(self, send, sb, recv, cap, rb):
        total = 0
        for p in range(self.world):
            n = int(sb[p]) & COUNT_MASK
            rb[p] = int(sb[p])
            total += n
        if total > cap:
            raise RuntimeError("receive capacity")
        if total:
            C.memset(recv, 0, total)


class ThreadExchange:
    """W shards in one process: rank r's callback deposits its blocks, waits for every rank, takes its own."""

    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.blocks = [None] * world
        self.ends = []

    def endpoint(self, rank):
        ex = self

        class _End(_HostExchange):
            def _run(self, send, sb, recv, cap, rb):
                W = ex.world
                words = [int(sb[q]) for q in range(W)]
                counts = [w & COUNT_MASK for w in words]
                data = C.string_at(send, sum(counts)) if sum(counts) else b""
                ex.blocks[rank] = (counts, words, data)
                ex.barrier.wait(timeout=300)
                parts = []
                for p in range(W):
                    cnts, wds, dat = ex.blocks[p]
                    off = sum(cnts[:rank])
                    parts.append(dat[off:off + cnts[rank]])
                    rb[p] = wds[rank]
                buf = b"".join(parts)
                if len(buf) > cap:
                    raise RuntimeError("receive capacity")
                if buf:
                    C.memmove(recv, buf, len(buf))
                ex.barrier.wait(timeout=300)

        e = _End()
        self.ends.append(e)
        return e


class ShardedCluster(SimulatedCluster):
    """One shard of a row-sharded simulation (swim_create_sharded)."""

    def __init__(self, lib, cfg: SimConfig, rank, world, transport=_abi.TRANSPORT_HOST, exchange=None,
                 rccl_id=None, chunk_cap=0):
        _abi.bind_shard(lib)
        self.lib = lib
        self.cfg = cfg
        self.n = cfg.n_members
        self.rank, self.world = rank, world
        self.exchange = exchange
        self._h = C.c_void_p()
        spec = _abi.SwimShardSpec()
        spec.rank, spec.world, spec.transport, spec.chunk_cap = rank, world, transport, chunk_cap
        if transport == _abi.TRANSPORT_RCCL:
            if rccl_id is None or len(rccl_id) != 128:
                raise ValueError("RCCL transport needs the 128-byte unique id of rank 0")
            for i, b in enumerate(rccl_id):
                spec.rccl_id[i] = b
        else:
            if exchange is None:
                raise ValueError("HOST transport needs an exchange object")
            spec.exchange = exchange.callback()
        self._spec = spec
        a = cfg.to_abi()
        rc = lib.swim_create_sharded(C.byref(a), C.byref(spec), C.byref(self._h))
        if rc != 0:
            raise SwimError(f"swim_create_sharded failed rc={rc} (rank {rank} of {world})")
        self._groups = {cfg.cluster.syncGroup: 0}
        lo, hi = C.c_uint32(), C.c_uint32()
        self._ck(lib.swim_shard_range(self._h, C.byref(lo), C.byref(hi)), "swim_shard_range")
        self.lo, self.hi = lo.value, hi.value

    def _ck(self, rc, what):
        if rc != 0 and self.exchange is not None and getattr(self.exchange, "error", None) is not None:
            raise SwimError(f"{what} failed rc={rc}: exchange error {self.exchange.error!r}")
        super()._ck(rc, what)

    def owns(self, m):
        return self.lo <= m < self.hi


class ThreadShardGroup:
    """W shards of one simulation driven from one process (one thread per shard, ThreadExchange transport).

    It offers the SimulatedCluster interface over the whole member range, so parity tests diff it against the
    oracle exactly like a single-GPU handle: hashes and counters are summed over the shards (each shard leaves the
    other shards' observers zero), event streams are merged in (tick, observer, seq) order, and per-observer
    readback goes to the owning shard."""

    def __init__(self, lib, cfg: SimConfig, world, chunk_cap=0):
        self.n = cfg.n_members
        self.world = world
        # RUMOR mode shards the gossips instead of the observers: every shard runs every member
        self.slots = cfg.mode == _abi.MODE_RUMOR
        self._evcount = {}
        self.ex = ThreadExchange(world)
        self.shards = [ShardedCluster(lib, cfg, r, world, _abi.TRANSPORT_HOST, self.ex.endpoint(r), chunk_cap=chunk_cap)
                       for r in range(world)]

    def _owner(self, m):
        for s in self.shards:
            if s.owns(m):
                return s
        raise IndexError(m)

    def _all(self, fn):
        errs = [None] * self.world

        def run(i):
            try:
                fn(self.shards[i])
            except BaseException as e:  # noqa: BLE001
                errs[i] = e
                self.ex.barrier.abort()

        ts = [threading.Thread(target=run, args=(i,)) for i in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for e in errs:
            if e is not None and not isinstance(e, threading.BrokenBarrierError):
                raise e
        for e in errs:
            if e is not None:
                raise e

    def step(self, ticks=1):
        self._all(lambda s: s.step(ticks))

    def run_periods(self, n):
        self._all(lambda s: s.run_periods(n))

    @property
    def tick(self):
        return self.shards[0].tick

    def kill(self, m):
        for s in self.shards:
            s.kill(m)

    def set_default_loss(self, pct):
        for s in self.shards:
            s.set_default_loss(pct)

    def partition(self, g):
        for s in self.shards:
            s.partition(g)

    def unblock_all(self):
        for s in self.shards:
            s.unblock_all()

    def leave(self, m):
        for s in self.shards:
            s.leave(m)

    def spread_gossip(self, m, payload):
        for s in self.shards:
            s.spread_gossip(m, payload)

    def join(self, m, seeds=()):
        for s in self.shards:
            s.join(m, seeds)

    def set_link_loss(self, src, dst, pct):
        for s in self.shards:
            s.set_link_loss(src, dst, pct)

    def set_default_link_settings(self, loss, mean_delay_ms):
        for s in self.shards:
            s.set_default_link_settings(loss, mean_delay_ms)

    def set_link_settings(self, src, dst, loss, mean_delay_ms):
        for s in self.shards:
            s.set_link_settings(src, dst, loss, mean_delay_ms)

    def emulator_counters(self):
        """Every member's (sent, lost) NetworkEmulator counters: each shard counted the sends it evaluated (its issuers'
        FD / SYNC / metadata messages, the gossip sends to its targets), so the shards' arrays add up."""
        out = self.shards[0].emulator_counters().copy()
        for s in self.shards[1:]:
            out += s.emulator_counters()
        return out

    def block(self, src, *dsts):
        for s in self.shards:
            s.block(src, *dsts)

    def unblock(self, src, *dsts):
        for s in self.shards:
            s.unblock(src, *dsts)

    def update_incarnation(self, m):
        for s in self.shards:
            s.update_incarnation(m)

    def set_member_config(self, m, cc):
        for s in self.shards:  # replicated on every shard, like the network settings
            s.set_member_config(m, cc)

    def update_metadata(self, m):
        for s in self.shards:
            s.update_metadata(m)

    def state_hash(self):
        h = self.shards[0].state_hash().copy()
        for s in self.shards[1:]:
            if self.slots:  # replicated row / lists / scalars; events and held gossips are per-shard sums
                part = s.state_hash().reshape(-1, _abi.HASH_WORDS)
                hv = h.reshape(-1, _abi.HASH_WORDS)
                hv[:, 3] += part[:, 3]
                hv[:, 4] += part[:, 4]
            else:
                h += s.state_hash()  # disjoint observer rows; the rest are zero
        return h

    def counters(self):
        cs = [s.counters() for s in self.shards]
        return {k: (sum(c[k] for c in cs) if k != "tick" else cs[0][k]) for k in cs[0]}

    def events(self):
        ev = [e for s in self.shards for e in s.events()]
        if not self.slots:
            ev.sort(key=lambda e: (e.tick, e.observer, e.seq))
            return ev
        # slot-sharded: an observer's events of one tick come from several shards; P4 order is the gossip id
        ev.sort(key=lambda e: (e.tick, e.observer, e.member, e.gossipCounter))
        out = []
        for e in ev:
            seq = self._evcount.get(e.observer, 0)
            self._evcount[e.observer] = seq + 1
            out.append(dataclasses.replace(e, seq=seq))
        return out

    def row(self, m):
        return self._owner(m).row(m)

    def lists(self, m):
        return self._owner(m).lists(m)

    def gossips(self, m):
        if self.slots:
            return sorted(g for s in self.shards for g in s.gossips(m))
        return self._owner(m).gossips(m)

    def close(self):
        for s in self.shards:
            s.close()
