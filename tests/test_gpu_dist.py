"""RCCL path on the real GPU (world 1): the DP step with its all-reduce captured in a HIP graph, and the
overlapped bucketed backward (side stream, forced with overlap_chunks) captured the same way."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_nccl_dp_step_in_graph_matches_fused(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29000 + os.getpid() % 1000))
    code = ("import sys; sys.path.insert(0, %r); from tests.dist_workers import nccl_graph_worker; "
            "nccl_graph_worker(%r)" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), str(tmp_path)))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    z = np.load(tmp_path / "nccl.npz")
    np.testing.assert_array_equal(z["a"], z["b"])
    np.testing.assert_array_equal(z["a1"], z["b1"])
    for H in (1024, 4096):  # bucketed + side-stream RCCL backward in the graph == the fused step
        assert float(z[f"bucketed_rel_{H}"]) <= 1e-6, (H, float(z[f"bucketed_rel_{H}"]))
