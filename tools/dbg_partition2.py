import sys, ctypes as C
sys.path.insert(0, "scalecube-cluster_amd")
import numpy as np
from swimhip import _abi, SimConfig, ClusterConfig, SimulatedCluster, engine, SwimError
lib = engine()
n = 48
def run(rec, chunk, label):
    e = SimulatedCluster(lib, SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, n - 1]), record_events=rec))
    e.partition(np.array([0] * (n // 2) + [1] * (n // 2), dtype=np.uint32))
    try:
        while e.tick < 350:
            e.step(chunk)
        h = e.state_hash()
        print(label, "ok", e.tick, hex(int(h.sum())), flush=True)
    except SwimError as ex:
        print(label, "ERR tick", e.tick, ex, flush=True)
    return e
keep = []
keep.append(run(False, 1, "a"))
keep.append(run(True, 25, "b"))
keep.append(run(True, 25, "c"))
big = SimulatedCluster(lib, SimConfig(n_members=300, record_events=True)); big.set_default_loss(5); big.step(200); keep.append(big)
keep.append(run(True, 25, "d"))
keep.append(run(False, 1, "e"))
