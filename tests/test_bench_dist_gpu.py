"""bench.py's world > 1 branch end to end: the driver's scaling run launches
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``; this runs that command at N=2 on the
box's one GPU with the test-only overrides AVT_BENCH_BACKEND=gloo and AVT_BENCH_ONE_DEVICE=1 (RCCL needs one device
per rank; both ranks share cuda:0, as tests/test_ddp_gpu.py does).  It must print one JSON line with configs[2]'s
sharding (global 256 -> 128 per GPU, strong scaling) and a roofline measured on eager launches."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(400)
def test_bench_two_ranks_prints_one_valid_line():
    env = dict(os.environ, AVT_BENCH_BACKEND="gloo", AVT_BENCH_ONE_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--traffic", "off", "--no-peaks"]
    r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=360)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    print(json.dumps({k: rec[k] for k in ("value", "ms_per_step", "n_gpus", "scaling", "backend")}))
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong" and rec["backend"] == "gloo"
    assert rec["config"]["per_gpu_batch"] == 128 and rec["config"]["global_batch"] == 256
    assert rec["config"]["parallelism"] == "dp2"
    assert math.isfinite(rec["value"]) and rec["value"] > 0 and math.isfinite(rec["loss"])
    roof = rec["roofline"]
    assert roof["launches"] > 0 and roof["achieved"] > 0 and roof["frac"] > 0, roof
    assert {"fwd", "dgrad", "wgrad"} <= set(roof["per_kind"]), roof["per_kind"]
    assert rec["avt_env"].get("AVT_BENCH_BACKEND") == "gloo"
