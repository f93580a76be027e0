"""Failure detection, structured logging and checkpoint/resume of the training CLI (CPU, gloo)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--backend", "torch", "--data", "synthetic", "--num-train", "3000", "--num-test", "500", "-n", "32",
         "-b", "400", "-l", "0.01"]


def _env():
    return dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")


def test_injected_fault_takes_the_job_down(tmp_path):
    port = 29700 + os.getpid() % 200
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "cme213_sp18_amd.train", *SMALL,
           "-e", "4", "--fault-inject", "1:3", "--comm-timeout", "30", "--outdir", str(tmp_path / "out")]
    t = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=300, cwd=str(tmp_path))
    el = time.time() - t
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-2000:]
    assert "injected fault on rank 1 at step 3" in out, out[-2000:]
    assert el < 120, f"job took {el:.0f}s to fail"


def test_json_log_periodic_checkpoint_and_resume(tmp_path):
    ck, lg = tmp_path / "ckpt", tmp_path / "log.jsonl"
    base = [sys.executable, "-m", "cme213_sp18_amd.train", *SMALL, "--outdir", str(tmp_path / "out"),
            "--ckpt-dir", str(ck), "--log-json", str(lg)]
    r = subprocess.run(base + ["-e", "3", "--ckpt-every", "1", "-p", "5"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    ev = [json.loads(l) for l in open(lg)]
    kinds = [e["event"] for e in ev]
    assert kinds[0] == "config" and kinds[-1] == "summary"
    assert kinds.count("checkpoint") == 2 and "loss" in kinds
    meta = json.load(open(ck / "meta.json"))
    assert meta["epochs"] == 3 and meta["iter"] == 3 * 7  # 2700 train columns / 400 per batch
    r2 = subprocess.run(base + ["-e", "1", "--resume", str(ck)], capture_output=True, text=True, env=_env(),
                        timeout=300)
    assert r2.returncode == 0, r2.stdout[-2000:] + r2.stderr[-2000:]
    assert "Resumed from" in r2.stdout
    assert json.load(open(ck / "meta.json"))["epochs"] == 4
