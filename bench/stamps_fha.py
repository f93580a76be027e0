#!/usr/bin/env python3
"""Timeline of the all-gather forward + head launch (mlp_fwd1_head_ag) from s_memrealtime stamps (100 MHz):
per workgroup entry -> GEMM + z2 partial published -> all tm workgroups of its column tile arrived ->
dZ1 stored.  Diagnostic.

    python bench/stamps_fha.py [--n 800] [--hidden 100]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the two-launch kernels' stamps exist only in the diagnostics library (_hip_diag: `python -m cme213_sp18_amd._build
# --diag`, built on first use)
os.environ.setdefault("CME_DIAG", "1")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=800)
    ap.add_argument("--hidden", type=int, default=100)
    ap.add_argument("--xcd-rows", type=int, default=None, help="MlpStep.xcd_rows (default: the engine's)")
    ap.add_argument("--warm-fwd", action="store_true",
                    help="one extra forward before the stamped one: W1 last READ, not written, by the previous launch")
    ap.add_argument("--head-dw2", type=int, default=None, help="MlpStep.head_dw2 (default: the engine's)")
    ap.add_argument("--store-a1", type=int, default=None, help="MlpEngine.set_store_a1 (default: the engine's)")
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import MlpEngine
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(4000, seed=0)
    nn = NeuralNetwork([784, a.hidden, 10])
    e = MlpEngine(nn.H, dtype="f32", max_cols=a.n, device="cuda", path="split3")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    step = e._hip_step()
    assert step.fh_allgather == 1
    if a.xcd_rows is not None:
        step.xcd_rows = a.xcd_rows
    if a.head_dw2 is not None:
        step.head_dw2 = a.head_dw2
    if a.store_a1 is not None:
        e.set_store_a1(bool(a.store_a1))
    st = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(4096 * 4, dtype=torch.int64, device="cuda")
    wbuf = torch.zeros(4096 * 8 * 4, dtype=torch.int64, device="cuda")
    pct = lambda v: [round(float(np.percentile(v, q)), 3) for q in (0, 50, 90, 100)]  # noqa: E731

    def per_wg(wb, t0):
        g = wb.view(-1, 8, 4).cpu().numpy().astype(np.int64)
        g = g[(g[:, :, 0] > 0).all(axis=1)]
        r = (g - t0) * 10.0 / 1000.0
        return {"wg_entry_spread": pct(r[:, :, 0].max(1) - r[:, :, 0].min(1)),
                "wg_first_entry_to_last_kloop": pct(r[:, :, 1].max(1) - r[:, :, 0].min(1))}
    for rep in range(4):
        for _ in range(20):
            step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 3)
        if a.warm_fwd:
            step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 1)
        torch.cuda.synchronize()
        buf.zero_()
        wbuf.zero_()
        step.stamps = buf.data_ptr()
        step.hstamps = wbuf.data_ptr()  # per wave of the GEMM tile (mma_tile.h wsk_tile)
        step.run(0, a.n, 1.0 / a.n, 1e-4, 0.0, 1, 0, st, 1)
        step.stamps = step.hstamps = 0
        torch.cuda.synchronize()
        s = buf.view(-1, 4).cpu().numpy().astype(np.int64)
        s = s[s[:, 0] > 0]
        t0 = s[:, 0].min()
        rel = (s - t0) * 10.0 / 1000.0
        w = wbuf.view(-1, 4).cpu().numpy().astype(np.int64)
        w = w[w[:, 0] > 0]
        wr = (w - t0) * 10.0 / 1000.0
        print(json.dumps({"head_dw2": int(step.head_dw2), "store_a1": int(step.store_a1), "wgs": int(len(s)), "entry": pct(rel[:, 0]), "published": pct(rel[:, 1]),
                          "all_arrived": pct(rel[:, 2]), "wait": pct(rel[:, 2] - rel[:, 1]), "end": pct(rel[:, 3]),
                          "wave_entry": pct(wr[:, 0]), "wave_kloop": pct(wr[:, 1]), "wave_reduced": pct(wr[:, 2]),
                          "wave_epilogue": pct(wr[:, 3]), "kloop_dur": pct(wr[:, 1] - wr[:, 0]),
                          # per workgroup (8 waves): first -> last wave entry, and first wave entry -> last K-loop end
                          **per_wg(wbuf, t0)}))
        if rep == 3:  # per wave index, relative to its workgroup's entry stamp (wave 0, thread 0): median / p90
            g = wbuf.view(-1, 8, 4).cpu().numpy().astype(np.int64)
            wg = buf.view(-1, 4).cpu().numpy().astype(np.int64)
            nb = min(g.shape[0], wg.shape[0])
            g, wg = g[:nb], wg[:nb]
            keep = (wg[:, 0] > 0) & (g[:, :, 0] > 0).all(axis=1)
            g, wg = g[keep], wg[keep]
            rel_w = (g - wg[:, None, 0:1]) / 100.0
            print(json.dumps({"warm_fwd": a.warm_fwd, "per_wave": {str(w): {"entry": pct(rel_w[:, w, 0])[1:3], "kloop_end": pct(rel_w[:, w, 1])[1:3],
                                                    "kloop_dur": pct(rel_w[:, w, 1] - rel_w[:, w, 0])[1:3]}
                                           for w in range(8)},
                              "wg_published": pct((wg[:, 1] - wg[:, 0]) / 100.0)[1:3],
                              "wg_arrived": pct((wg[:, 2] - wg[:, 0]) / 100.0)[1:3],
                              "wg_end": pct((wg[:, 3] - wg[:, 0]) / 100.0)[1:3]}), flush=True)
        # per column tile: its last publication -> each of its workgroups' arrival (the hand-off's own latency)
        tm_ = (a.hidden + 15) // 16
        allv = buf.view(-1, 4).cpu().numpy().astype(np.int64)
        byct = {}
        for b in range(allv.shape[0]):
            if allv[b, 0] <= 0:
                continue
            xcd, slot = b & 7, b >> 3
            ct = slot if step.xcd_rows else xcd + 8 * (slot // tm_)
            byct.setdefault(ct, []).append(allv[b])
        lat, first = [], []
        for ct, v in byct.items():
            v = np.array(v)
            lastpub = v[:, 1].max()
            lat += list((v[:, 2] - lastpub) / 100.0)
            first.append((v[:, 2].min() - lastpub) / 100.0)
        # per row tile (= XCD under xcd_rows): when its workgroups published (GEMM + epilogue done)
        byrt, byrt_e, byrt_k = {}, {}, {}
        wall = wbuf.view(-1, 8, 4).cpu().numpy().astype(np.int64)
        for b in range(allv.shape[0]):
            if allv[b, 0] <= 0:
                continue
            xcd, slot = b & 7, b >> 3
            rt = xcd if step.xcd_rows else slot % tm_
            byrt.setdefault(rt, []).append((allv[b, 1] - t0) / 100.0)
            byrt_e.setdefault(rt, []).append((allv[b, 0] - t0) / 100.0)
            if b < wall.shape[0] and (wall[b, :, 1] > 0).all():
                byrt_k.setdefault(rt, []).append((wall[b, :, 1].max() - t0) / 100.0)
        print(json.dumps({"handoff_after_last_publish": pct(lat), "first_arrival_after_last_publish": pct(first),
                          "published_by_row_tile": {str(k): pct(v) for k, v in sorted(byrt.items())},
                          "entry_by_row_tile": {str(k): pct(v) for k, v in sorted(byrt_e.items())},
                          "kloop_end_by_row_tile": {str(k): pct(v) for k, v in sorted(byrt_k.items())}}),
              flush=True)
        if rep == 3:  # per column tile (XCD-grouped grid: block b -> xcd b & 7, slot b >> 3, ct = xcd + 8 (slot // tm))
            tm = (a.hidden + 15) // 16
            allv = buf.view(-1, 4).cpu().numpy().astype(np.int64)
            per = {}
            for b in range(allv.shape[0]):
                if allv[b, 0] <= 0:
                    continue
                ct = (b & 7) + 8 * ((b >> 3) // tm)
                per.setdefault(ct, []).append(((allv[b, 0] - t0) / 100.0, (allv[b, 3] - t0) / 100.0))
            print(json.dumps({str(ct): {"last_entry": round(max(e for e, _ in v), 2), "last_end": round(max(x for _, x in v), 2)}
                              for ct, v in sorted(per.items())}), flush=True)


if __name__ == "__main__":
    main()
