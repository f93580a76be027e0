"""One command, N ranks: ``bench.py --gpus N`` and ``python -m cme213_sp18_amd.train --gpus N`` start their
ranks themselves when no launcher did (the reference's ``mpirun -np 4 ./main -g 2``, fpcode/run.sh:39), check
that the job really is N ranks on N distinct devices, and refuse -- non-zero exit, no record -- otherwise.
Also: a resumed run continues the iteration counter (loss lines, -d diff rows; fpcode/neural_network.cpp:
267-275, 543-553).  CPU only: gloo ranks, the torch backend."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "CME_SHARED_GPU")}
    env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS="2", **kw)
    return env


def _records(stdout: str):
    out = []
    for line in stdout.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                out.append(json.loads(line))
            except json.JSONDecodeError:
                pass
    return out


def test_bench_self_launches_n_ranks(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "torch",
                        "--steps", "3", "--warmup", "1", "--train-size", "3200"],
                       cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    recs = _records(r.stdout)
    assert len(recs) == 1, r.stdout  # rank 0 only
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["config"]["ranks_seen"] == 2 and rec["config"]["parallelism"] == "dp2"
    # no --scaling flag: the metric's own config -- global batch 800 split over the ranks (fpcode/run.sh:39,
    # neural_network.cpp:458) -- and the weak-scaling run as a labelled secondary sub-record
    assert rec["scaling"] == "strong" and rec["config"]["global_batch"] == 800, rec
    assert rec["config"]["per_gpu_batch"] == 400
    weak = rec["weak"]
    assert weak["global_batch"] == 1600 and weak["per_gpu_batch"] == 800 and weak["value"] > 0, weak
    assert rec["config"]["devices_distinct"] is True
    assert rec["config"]["allreduce_us"] > 0 and rec["config"]["allreduce_bytes"] > 300_000
    assert rec["config"]["allreduce_pred_us"] > 0  # the cost model's prediction beside the measurement
    assert rec["steps"] == 3 and rec["value"] > 0


def test_bench_weak_primary_with_strong_secondary(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "torch",
                        "--scaling", "weak", "--steps", "2", "--warmup", "1", "--train-size", "3200"],
                       cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = _records(r.stdout)[0]
    assert rec["scaling"] == "weak" and rec["config"]["global_batch"] == 1600
    assert rec["strong"]["global_batch"] == 800 and rec["strong"]["per_gpu_batch"] == 400


def test_bench_refuses_more_gpus_than_visible(tmp_path):
    """The hip backend with more ranks than GPUs (here: none visible): exit non-zero, print no record."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2",
                        "--warmup", "1"], cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not _records(r.stdout), r.stdout
    assert "GPU" in r.stderr


def test_bench_refuses_rank_count_mismatch(tmp_path):
    """Launched as 2 ranks but asked for --gpus 3: every rank refuses, no record."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29671", os.path.join(ROOT, "bench.py"),
                        "--gpus", "3", "--backend", "torch", "--steps", "2", "--warmup", "1", "--train-size", "3200"],
                       cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not _records(r.stdout), r.stdout
    assert "2 rank" in r.stderr


def test_train_cli_self_launches_n_ranks(tmp_path):
    log = tmp_path / "run.jsonl"
    r = subprocess.run([sys.executable, "-m", "cme213_sp18_amd.train", "--preset", "cpu_plumbing", "-n", "16",
                        "-e", "1", "--num-train", "1600", "--num-test", "100", "--gpus", "2", "--log-json", str(log),
                        "--outdir", str(tmp_path / "Outputs")],
                       cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    ev = [json.loads(line) for line in log.read_text().splitlines()]
    cfg = next(e for e in ev if e.get("event") == "config")
    assert cfg["world"] == 2 and cfg["ranks_seen"] == 2 and cfg["devices_distinct"] is True
    assert any(e.get("event") == "summary" for e in ev)


def test_resume_continues_iteration_counter(tmp_path):
    """-s -d -p 1 for one epoch with a checkpoint, then --resume for one more: the loss lines and the
    CpuGpuDiff.txt rows of the second run are iterations 2 and 3 (appended, not truncated), and the CPU
    oracle's snapshots carry the same numbers so the diff still compares like with like."""
    common = [sys.executable, "-m", "cme213_sp18_amd.train", "--preset", "cpu_plumbing", "-n", "16",
              "--num-train", "1600", "--num-test", "100", "-s", "-d", "-p", "1", "-e", "1",
              "--outdir", str(tmp_path / "Outputs")]
    r1 = subprocess.run(common + ["--ckpt-dir", str(tmp_path / "ckpt")], cwd=tmp_path, env=_env(),
                        capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stderr[-3000:]
    meta = json.loads((tmp_path / "ckpt" / "meta.json").read_text())
    assert meta["iter"] == 2 and meta["epochs"] == 1
    r2 = subprocess.run(common + ["--resume", str(tmp_path / "ckpt")], cwd=tmp_path, env=_env(),
                        capture_output=True, text=True, timeout=600)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert "Loss at iteration 2 of epoch" in r2.stdout and "Loss at iteration 0 of epoch" not in r2.stdout
    rows = (tmp_path / "Outputs" / "CpuGpuDiff.txt").read_text().splitlines()
    its = [int(line.split()[0]) for line in rows if line.split() and line.split()[0].isdigit()]
    assert its == [0, 1, 2, 3], rows
    assert (tmp_path / "Outputs" / "CPUmats" / "SequentialW0-3.mat").exists()
    out = json.loads(r2.stdout.strip().splitlines()[-1])
    assert out["correct"] is True
