#!/usr/bin/env python3
"""Predicted strong-scaling curve of the headline (global batch 800 over N ranks, n = 800 / N per rank) from
measured one-GPU per-rank steps (a bench/kbench.py jsonl: step_fused_us, step_xgmi1_us, step_push1_us by n) and the
all-reduce cost model (cme213_sp18_amd.parallel.trainer.CostModel; bench.py measures its constants at N > 1 on the
node and records them as cost_model_measured).  Stated model, per step at N ranks:

  pull (the one-shot fused into the weight-gradient launch):  step_xgmi1(n) + 3 hops + S / B
      (a flag one way, then every rank READS each peer's tile: a round trip, S bytes over each link)
  push (the owner-tile form, XgmiFuse::push):                   step_push1(n) + 2 hops + 4 S / (N B)
      (the gradient tile one way to its owner, the update one way back; 2 S / N payload bytes per link each way,
      twice that with the 8-byte {value, tag} granules)

S = the fp32 gradient bucket (318,208 B at 784-100-10), B = one link's rate, hop = one one-way xGMI latency
(--hop-us; a planning number: nothing here has crossed two GPUs).  N = 1 is the one-process step (step_walk_us,
the training form's consecutive batches).  Prints one JSON line per N and form.

    python bench/predict_scaling.py profiles/r5/kbench_headline.jsonl [--hop-us 1.0] [--link-gbps 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

S_BYTES = 79_552 * 4  # the flat [W1|b1|W2|b2|status] fp32 bucket at 784-100-10 (64-element aligned segments)


def predict(rows: dict[int, dict], hop_us: float, link_gbps: float, batch: int = 800) -> list[dict]:
    bw = link_gbps * 1e3  # bytes per us
    out = []
    for N in (1, 2, 4, 8):
        n = batch // N
        r = rows.get(n)
        if r is None:
            continue
        if N == 1:
            us = r.get("step_walk_us") or r["step_fused_us"]
            out.append({"N": 1, "n": n, "form": "one process", "us_per_step": round(us, 2),
                        "images_per_s": round(batch / us * 1e6 / 1e6, 1)})
            continue
        forms = {"pull": r["step_xgmi1_us"] + 3 * hop_us + S_BYTES / bw,
                 "push": r.get("step_push1_us", float("nan")) + 2 * hop_us + 4 * S_BYTES / (N * bw)}
        for f, us in forms.items():
            out.append({"N": N, "n": n, "form": f, "us_per_step": round(us, 2),
                        "images_per_s": round(n * N / us * 1e6 / 1e6, 1)})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("kbench_jsonl")
    ap.add_argument("--hop-us", type=float, default=1.0)
    ap.add_argument("--link-gbps", type=float, default=64.0)
    a = ap.parse_args(argv)
    rows = {}
    with open(a.kbench_jsonl) as f:
        text = f.read().strip()
    recs = json.loads(text) if text.startswith("[") else [json.loads(l) for l in text.splitlines() if l.startswith("{")]
    for r in recs:
        if r.get("path", "").startswith("split3") and r.get("H") == 100:
            rows[int(r["n"])] = r
    for p in predict(rows, a.hop_us, a.link_gbps):
        print(json.dumps({**p, "hop_us": a.hop_us, "link_GBps": a.link_gbps, "images_unit": "M/s"}))


if __name__ == "__main__":
    main()
