"""Debugging aid: replay one fuzz schedule on engine and oracle, compare after every tick from a given tick on, and
print one member's scalar fields (swimdbg_scalars) around the first divergence.
usage: python tools/dbg_scalars.py SEED MEMBER FROM_TICK"""
import ctypes as C
import sys
sys.path.insert(0, "scalecube-cluster_amd"); sys.path.insert(0, "tests")
import parity_util
import test_gpu_fuzz as F
from swimhip import _abi, engine
from swimhip.cluster import SimulatedCluster

seed, mem, t0 = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cfg, acts = F.schedule(seed)
o, e = SimulatedCluster(_abi.load("oracle/liboracle_swimref.so"), cfg), SimulatedCluster(engine(), cfg)


def sc(c):
    fn = c.lib.swimdbg_scalars
    fn.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 6)()
    fn(c._h, mem, out)
    return list(out)


orig = parity_util.run_lockstep


def lockstep(o, e, ticks, chunk, where="", events=True):
    for _ in range(ticks):
        if o.tick < t0:
            orig(o, e, 1, 1, where, False) if False else (o.step(1), e.step(1))
            continue
        o.step(1), e.step(1)
        a, b = sc(o), sc(e)
        print(o.tick, a, b, "" if a == b else "<<<", flush=True)
        if a != b:
            raise AssertionError("diverged")


F.run_lockstep = lockstep
try:
    F.play(o, e, acts, f"seed {seed}", cfg.n_dormant)
    print("seed", seed, "OK", o.tick)
except AssertionError as ex:
    print("seed", seed, "FAIL", str(ex)[:2000])
