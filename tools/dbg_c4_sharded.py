"""Debugging aid: sharded (W=2) vs oracle on the c4_small golden scenario, tick by tick after the heal; prints the
first divergence with the member's row / gossip differences."""
import sys
import numpy as np
sys.path.insert(0, "scalecube-cluster_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden")
from swimhip import _abi, engine
from swimhip.cluster import SimulatedCluster
from swimhip.shard import ThreadShardGroup
from scenarios import SCENARIOS
from parity_util import first_diff
W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
def load_any(path):  # an older build may lack newer entry points
    import ctypes as C
    lib = C.CDLL(path, mode=C.RTLD_LOCAL)
    for name, (res, args) in _abi.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    return lib


LIB = load_any(sys.argv[2]) if len(sys.argv) > 2 else engine()
cfg, acts = SCENARIOS["c4_small"]()
o = SimulatedCluster(_abi.load("oracle/liboracle_swimref.so"), cfg)
e = ThreadShardGroup(LIB, cfg, W) if W > 1 else SimulatedCluster(LIB, cfg)
for c in (o, e): c.partition(np.array(acts[0][1], dtype=np.uint32))
for c in (o, e): c.run_periods(34)
for c in (o, e): c.unblock_all()
for t in range(60):
    for c in (o, e): c.step(1)
    d = first_diff(o.state_hash(), e.state_hash())
    co, ce = o.counters(), e.counters()
    cd = {k: (co[k], ce[k]) for k in ("record_compares", "row_writes", "messages", "gossip_messages", "events", "gossips_created") if co[k] != ce[k]}
    if d or cd:
        print("tick", o.tick, "first diff", d, "counters", cd)
        m = d[0] if d else 10
        go, ge = set(o.gossips(m)), set(e.gossips(m))
        print(" gossips oracle-only", sorted(go - ge)[:8], "engine-only", sorted(ge - go)[:8])
        ro, re_ = o.row(m), e.row(m)
        print(" row diffs", [(int(s), hex(int(ro[s])), hex(int(re_[s]))) for s in np.nonzero(ro != re_)[0][:8]])
        break
print("done", o.tick)
