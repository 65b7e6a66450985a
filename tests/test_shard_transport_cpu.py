"""The N>1 host path on CPU: the gloo-driven SWIM_TRANSPORT_HOST exchange (swimhip.shard.GlooExchange) between
world_size 2 and 3 processes, called exactly as libswimhip calls it (ctypes thunk, host buffers, rank-ordered
blocks), plus the shard ranges the library uses. No GPU is touched."""
import ctypes as C
import os
import socket

import pytest
import torch.multiprocessing as mp

from swimhip.shard import GlooExchange, ThreadExchange, shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = GlooExchange()
        cb = ex.callback()
        # block for peer p: bytes (rank, p, i) for i < 3 + rank + p; nothing for itself
        blocks = [b"" if p == rank else bytes((rank * 16 + p * 4 + i) & 0xFF for i in range(3 + rank + p))
                  for p in range(world)]
        data = b"".join(blocks)
        send = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data.ljust(max(1, len(data)), b"\0"))
        sb = (C.c_uint64 * world)(*[len(b) for b in blocks])
        recv = (C.c_uint8 * 256)()
        rb = (C.c_uint64 * world)()
        rc = cb(None, C.cast(send, C.c_void_p), sb, C.cast(recv, C.c_void_p), 256, rb)
        got, off = [], 0
        for p in range(world):
            got.append(bytes(recv[off:off + rb[p]]))
            off += rb[p]
        want = [b"" if p == rank else bytes((p * 16 + rank * 4 + i) & 0xFF for i in range(3 + p + rank))
                for p in range(world)]
        q.put((rank, rc, got == want, repr(ex.error)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_all_to_all(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert [r[1] for r in res] == [0] * world, res
    assert all(r[2] for r in res), res


def test_thread_exchange_all_to_all():
    import threading
    world = 3
    ex = ThreadExchange(world)
    ends = [ex.endpoint(r) for r in range(world)]
    cbs = [e.callback() for e in ends]
    out = [None] * world

    def run(rank):
        blocks = [b"" if p == rank else bytes([rank, p]) * (1 + p) for p in range(world)]
        data = b"".join(blocks) or b"\0"
        send = (C.c_uint8 * len(data)).from_buffer_copy(data)
        sb = (C.c_uint64 * world)(*[len(b) for b in blocks])
        recv = (C.c_uint8 * 64)()
        rb = (C.c_uint64 * world)()
        assert cbs[rank](None, C.cast(send, C.c_void_p), sb, C.cast(recv, C.c_void_p), 64, rb) == 0
        got, off = [], 0
        for p in range(world):
            got.append(bytes(recv[off:off + rb[p]]))
            off += rb[p]
        out[rank] = got

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for r in range(world):
        assert out[r] == [b"" if p == r else bytes([p, r]) * (1 + r) for p in range(world)]


@pytest.mark.parametrize("n,w", [(64, 2), (300, 3), (100_000, 8), (50, 7), (1_000_000, 8)])
def test_shard_ranges_partition_members(n, w):
    r = [shard_range(n, w, i) for i in range(w)]
    assert r[0][0] == 0 and r[-1][1] == n
    assert all(r[i][1] == r[i + 1][0] for i in range(w - 1))
    assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
