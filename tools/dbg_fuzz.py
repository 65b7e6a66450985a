"""Debugging aid: replay one fuzz schedule (engine vs oracle) and print the first divergence.
usage: python tools/dbg_fuzz.py SEED [fast] [tick]   (tick: compare after every tick instead of the test's chunks)"""
import sys
sys.path.insert(0, "scalecube-cluster_amd"); sys.path.insert(0, "tests")
import parity_util
import test_gpu_fuzz as F
from swimhip import _abi, engine
from swimhip.cluster import SimulatedCluster

seed, fast, per_tick = int(sys.argv[1]), "fast" in sys.argv[2:], "tick" in sys.argv[2:]
orig = parity_util.run_lockstep
if per_tick:
    F.run_lockstep = lambda o, e, ticks, chunk, where="", events=True: orig(o, e, ticks, 1, where, events)
cfg, acts = F.schedule(seed, fast_sync=fast)
o, e = SimulatedCluster(_abi.load("oracle/liboracle_swimref.so"), cfg), SimulatedCluster(engine(), cfg)
try:
    F.play(o, e, acts, f"seed {seed}", cfg.n_dormant)
    print("seed", seed, "OK", o.tick)
except AssertionError as ex:
    print("seed", seed, "FAIL", str(ex)[:3000])
