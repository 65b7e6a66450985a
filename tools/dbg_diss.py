"""Debug: dissemination under 25% loss, oracle vs two engine instances, one tick at a time."""
import ctypes as C
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
import swimhip
from swimhip import SimConfig, _abi
from swimhip.cluster import SimulatedCluster

ora = _abi.load(ROOT / "oracle" / "liboracle_swimref.so")
eng = swimhip.engine()
for L in (ora, eng):
    L.swimdbg_scalars.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
names = ["cidCnt", "syncSeq", "gCounter", "nextSync", "fdPeriod", "gPeriod"]

def sc(c, m):
    out = (C.c_uint64 * 6)()
    c.lib.swimdbg_scalars(c._h, m, out)
    return list(out)

for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    cfg = SimConfig(n_members=50, record_events=True)
    o, e1, e2 = SimulatedCluster(ora, cfg), SimulatedCluster(eng, cfg), SimulatedCluster(eng, cfg)
    cs = (o, e1, e2)
    for c in cs:
        c.set_default_loss(25)
        c.step(5)
        c.update_incarnation(0)
    bad = False
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    for t in range(40 // chunk):
        for c in cs:
            c.step(chunk)
        h = [c.state_hash() for c in cs]
        for name, x in (("e1", h[1]), ("e2", h[2])):
            diff = np.argwhere(h[0] != x)
            if len(diff):
                m, w = diff[0]
                print(f"rep {rep} tick {o.tick}: {name} differs at member {m} word {w}; "
                      f"oracle {dict(zip(names, sc(o, m)))} engine {dict(zip(names, sc(cs[1 if name=='e1' else 2], m)))}", flush=True)
                bad = True
        if not np.array_equal(h[1], h[2]):
            print(f"rep {rep} tick {o.tick}: the two engine runs differ", flush=True)
        if bad:
            break
    print(f"rep {rep}: {'MISMATCH' if bad else 'ok'}", flush=True)
    for c in cs:
        c.close()
