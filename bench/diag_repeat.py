#!/usr/bin/env python3
"""Run-to-run determinism of one gradient step (sgd=False): the same step repeated on fresh engines in one
process must give BITWISE the same a1 / D / dZ1 / gradients every time.  Prints one JSON line per case with
the repeats that differed from the first and the first buffer (in step order) that differed.

    python bench/diag_repeat.py [--reps 20] [--cases 4096:160 1024:100]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cases", nargs="*", default=["4096:160", "4096:800", "1024:100", "100:800"])
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--mode", default="fresh", choices=["fresh", "same"],
                    help="fresh: a new engine per repeat; same: one engine re-running the same step")
    ap.add_argument("--pairs", type=int, default=None, help="MlpStep.u8_pairs (default: the engine's)")
    ap.add_argument("--allgather", type=int, default=None, help="MlpEngine.set_fh_allgather (default: on)")
    a = ap.parse_args(argv)
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    names = ("a1", "D", "dZ1", "gW1", "gb1", "gW2", "gb2")
    for case in a.cases:
        H, n = (int(v) for v in case.split(":"))
        x, y = synthetic_mnist(2 * n + 64, seed=3)
        nn = NeuralNetwork([784, H, 10])
        ref, bad = None, []

        def make():
            e = MlpEngine(nn.H, dtype=a.dtype, max_cols=n, device="cuda")
            e.set_params(*nn.params)
            e.load_dataset(x, y)
            if a.allgather is not None:
                e.set_fh_allgather(bool(a.allgather))
            if a.pairs is not None:
                e._hip_step().u8_pairs = a.pairs
            return e

        e = make()
        for r in range(a.reps):
            if a.mode == "fresh" and r:
                del e
                e = make()
            e.run(64, n, 1.0 / n, 1e-4, 0.0, sgd=False, with_loss=True)
            torch.cuda.synchronize()
            got = {k: getattr(e, k)[..., :n].clone() if k in ("a1", "D", "dZ1") else getattr(e, k).clone()
                   for k in names}
            if ref is None:
                ref = got
                continue
            diff = [k for k in names if not torch.equal(got[k], ref[k])]
            if diff:
                k = diff[0]
                d = (got[k].double() - ref[k].double()).abs()
                i = int(d.argmax())
                bad.append({"rep": r, "first": k, "all": diff, "max_abs": float(d.max()),
                            "where": [i // got[k].shape[-1], i % got[k].shape[-1]],
                            "count": int((d > 0).sum())})
        print(json.dumps({"H": H, "n": n, "dtype": a.dtype, "mode": a.mode, "pairs": a.pairs,
                          "allgather": a.allgather, "reps": a.reps, "bad": bad[:4], "n_bad": len(bad)}), flush=True)


if __name__ == "__main__":
    main()
