import sys, ctypes as C
sys.path.insert(0, "scalecube-cluster_amd")
import numpy as np
from swimhip import _abi, SimConfig, ClusterConfig, SimulatedCluster, engine, SwimError
lib = engine()
lib.swimdbg_read_log.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
n = 48
e = SimulatedCluster(lib, SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, n - 1])))
e.partition(np.array([0] * (n // 2) + [1] * (n // 2), dtype=np.uint32))
def dump(m):
    buf = (C.c_uint32 * 100000)(); lw = C.c_uint32(); f = C.c_uint32(); pos = C.c_uint32()
    lib.swimdbg_read_log(e._h, m, buf, 100000, C.byref(lw), C.byref(f), C.byref(pos))
    W = lw.value; F = f.value
    ents = sorted([(buf[i*(3+F)], buf[i*(3+F)+1], buf[i*(3+F)+2], [buf[i*(3+F)+3+j] for j in range(F)]) for i in range(W)])
    print("member", m, "LOGW", W, "pos", pos.value, "first", ents[:3], "last", ents[-3:])
try:
    for t in range(400):
        e.step(1)
except SwimError as ex:
    print("tick", e.tick, ex)
    info = [int(x) for x in str(ex).split("[info ")[1].split("]")[0].split()]
    print(info)
    dump(info[3]); dump(info[4])
