"""Debug: per-tick gossip send counts of oracle vs engine for a golden scenario, then the differing sends."""
import ctypes as C
import os
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
os.environ["SWIM_SEND_LOG"] = str(1 << 24)
os.environ["SWIMREF_SEND_LOG"] = "/tmp/oracle_sends.txt"
import swimhip
from swimhip import _abi
from swimhip.cluster import SimulatedCluster
from scenarios import SCENARIOS
name = sys.argv[1]
cfg, actions = SCENARIOS[name]()
o = SimulatedCluster(_abi.load(ROOT / "oracle" / "liboracle_swimref.so"), cfg)
e = SimulatedCluster(swimhip.engine(), cfg)
first = None
for what, arg in actions:
    for c in (o, e):
        if what == "partition":
            c.partition(np.array(arg, dtype=np.uint32))
        elif what == "unblock":
            c.unblock_all()
        elif what == "kill":
            c.kill(arg)
        elif what == "loss":
            c.set_default_loss(arg)
    if what != "periods":
        continue
    for _ in range(arg * 10):
        o.step(1)
        e.step(1)
        go, ge = o.counters()["gossip_messages"], e.counters()["gossip_messages"]
        if go != ge and first is None:
            first = o.tick - 1
            print("first differing tick", first, "oracle", go, "engine", ge, flush=True)
            break
    if first is not None:
        break
o.close()
lib = e.lib
lib.swimdbg_send_log.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_size_t)]
buf = (C.c_uint32 * (5 << 24))()
n = C.c_size_t()
print("rc", lib.swimdbg_send_log(e._h, buf, 1 << 24, C.byref(n)))
arr = np.frombuffer(buf, dtype=np.uint32, count=5 * n.value).reshape(-1, 5)
es = set((int(r[0]), int(r[1]), (int(r[3]) << 32) | int(r[2]), int(r[4])) for r in arr if r[0] == first)
os_ = set()
for line in open("/tmp/oracle_sends.txt"):
    k, m, g, t = map(int, line.split())
    if k == first:
        os_.add((k, m, g, t))
print("engine sends", len(es), "oracle sends", len(os_))
for x in sorted(os_ - es)[:20]:
    print("oracle-only", x[0], "sender", x[1], "gid", x[2] >> 32, x[2] & 0xFFFFFFFF, "target", x[3])
for x in sorted(es - os_)[:20]:
    print("engine-only", x[0], "sender", x[1], "gid", x[2] >> 32, x[2] & 0xFFFFFFFF, "target", x[3])
