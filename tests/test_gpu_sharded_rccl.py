"""Row sharding across processes (one per rank), as bench.py --gpus N runs it, on the single GPU of the test box.

RCCL: the ranks get distinct NCCL_HOSTID values so RCCL's duplicate-device check lets two ranks share the GPU; they
then exchange over RCCL's socket transport (on 8 GPUs the same library code runs over xGMI). HOST: the same shards
with the gloo-driven host transport. The worker checks every rank against the CPU oracle, bit-exact."""
import os
import subprocess
import sys
import time
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


# "full-xinl": the inline all-to-all block cut to 256 B (SWIM_CAPS xinl=), so most exchange-A regions overflow it: the
# speculative sharded batches halt on the overflow flag (XFLAG_OVER) and the host's send/recv group carries the rest
@pytest.mark.parametrize("transport,mode", [("host", "full"), ("rccl", "full"), ("rccl", "rumor"), ("rccl", "full-xinl")])
def test_two_process_shards(transport, mode, tmp_path):
    import torch  # noqa: F401  (pages torch in once, before two workers import it at the same time)
    procs, logs = [], []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT={"full": {"rccl": "29533", "host": "29534"}[transport], "rumor": "29535",
                                            "full-xinl": "29536"}[mode], NCCL_HOSTID=f"swimhost{r}",
                   NCCL_SOCKET_IFNAME="lo", GLOO_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        if mode == "full-xinl":
            env["SWIM_CAPS"] = "xinl=256"
        logdir = Path(os.environ.get("SWIM_TEST_LOGDIR", str(tmp_path)))
        logdir.mkdir(parents=True, exist_ok=True)
        log = open(logdir / f"{transport}_{mode}_rank{r}.log", "w")
        logs.append(log)
        procs.append(subprocess.Popen([sys.executable, "-u", str(ROOT / "tests" / "shard_rccl_worker.py"), transport, mode.split("-")[0]],
                                      env=env, stdout=log, stderr=subprocess.STDOUT))
    t0 = time.time()
    timed_out = False
    try:
        while any(p.poll() is None for p in procs):
            if time.time() - t0 > 240:
                timed_out = True
                break
            time.sleep(0.25)
            if int(time.time() - t0) % 10 == 0:
                print(f"[{transport}] {time.time() - t0:.0f}s", flush=True)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for f in logs:
            f.close()
    outs = [Path(f.name).read_text() for f in logs]
    assert not timed_out, "sharded workers did not finish in 240 s:\n" + "\n----\n".join(o[-3000:] for o in outs)
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} failed (rc {p.returncode}):\n{out[-4000:]}"
    assert "bit-exact" in outs[0], outs[0][-2000:]
    print(outs[0][-300:])
