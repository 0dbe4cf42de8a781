"""Tier C of the Hogwild O2 launch as a function of the contended-row set (the hot bitmap) and the
wavefronts in flight: held-out loss of one product launch against the committed sequential-oracle
fixture, and the launch time (HIP events), per setting.

Cases (tests/tierc_inputs.py): c5_1m (C5's kernel <4, true, 10> on a 1M-node graph of C5's
generator; fixture tierc_c5_1m_seq.json), c5 (C5 itself), c3_1m (the C3 bench launch, 1,048,576
walks).

Hot-set specs (comma-separated):
  share:X      rows holding >= X of the negative table (come_hot_rows; the product's rule at X =
               DEFAULT_HOT_P)
  all          every row hot (every update a float atomic)
  none         every row cold (plain stores)
  visit:X      share:DEFAULT_HOT_P plus the rows whose walk visits are >= X of the launch's positions
  upd:C        rows whose expected concurrent updaters per update (see come_amd.model.hot_rows_for)
               are >= C

    python scripts/tierc_hot_sweep.py --case c5_1m --hot share:5e-6,share:1e-6,all [--waves 0]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CASES = {
    "c5_1m": ("c5_1m_inputs", "tierc_c5_1m_seq.json", "C5_HYPER"),
    "c5": ("c5_inputs", "tierc_c5_seq.json", "C5_HYPER"),
    "c3_1m": ("c3_1m_inputs", "tierc_c3_1m_seq.json", "C3_HYPER"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="c5_1m", choices=sorted(CASES))
    ap.add_argument("--hot", default="share:5e-6")
    ap.add_argument("--waves", default="0")
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    import tierc_inputs as ti
    builder, fxname, hyper = CASES[args.case]
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", fxname)))
    dev = torch.device("cuda", 0)
    x = getattr(ti, builder)(**({"device": dev} if args.case == "c5" else {}))
    assert x.digest == fx["inputs_sha256"], "inputs differ from the fixture's"
    hp = getattr(ti, hyper)
    w, n, lr = hp["window"], hp["negative"], hp["lr"]
    ri, rp, rn = x.heldout(w, n)
    V = x.g.V
    tab = torch.from_numpy(x.table.view(np.int32)).to(dev)
    packed = tsi.pack_table(tab)
    walks = torch.from_numpy(x.train).to(dev)
    seeds = torch.from_numpy(x.seeds.view(np.int64)).to(dev)
    T = len(x.table)
    words = (V + 31) // 32
    print("case %s: V %d, d %d, walks %d, seq loss %.5f" % (
        args.case, V, x.node0.shape[1], walks.shape[0], fx["seq_loss"]), flush=True)

    def bitmap_of(mask):
        m = torch.zeros(words * 32, dtype=torch.bool, device=dev)
        m[:V] = mask
        b = m.view(words, 32).to(torch.int64) << torch.arange(32, device=dev, dtype=torch.int64)
        return b.sum(1).to(torch.int64).bitwise_and(0xFFFFFFFF).to(torch.int32)

    tcount = torch.bincount(tab.long(), minlength=V)[:V]
    wv = walks[walks >= 0].long()
    visits = torch.bincount(wv, minlength=V)[:V]
    positions = int(wv.numel())

    def hot_of(spec):
        if spec == "all":
            return bitmap_of(torch.ones(V, dtype=torch.bool, device=dev))
        if spec == "none":
            return None
        kind, val = spec.split(":")
        val = float(val)
        if kind == "share":
            return tsi.hot_rows(tab, V, max(1, int(val * T)))
        if kind == "visit":
            return bitmap_of((tcount >= int(tsi.DEFAULT_HOT_P * T)) | (visits >= val * positions))
        if kind == "upd":
            # expected updates of a row per launch: as a negative n x pairs x share, as a
            # positive / input 2w x visits; concurrent updaters ~ updates x waves / pairs
            pairs = 2 * w * positions
            upd = n * pairs * tcount.double() / T + 2 * w * visits.double() * 2
            waves = 4096
            return bitmap_of(upd * waves / pairs >= val)
        raise ValueError(spec)

    out = {"case": args.case, "seq_loss": fx["seq_loss"], "init_loss": fx["init_loss"],
           "points": []}
    for spec in args.hot.split(","):
        hot = hot_of(spec)
        nhot = V if spec == "all" else (0 if hot is None else int(
            sum(bin(int(v) & 0xFFFFFFFF).count("1") for v in hot.cpu().numpy())))
        for mw in [int(v) for v in args.waves.split(",")]:
            for _ in range(args.runs):
                node = torch.from_numpy(x.node0).to(dev)
                ctx = torch.zeros_like(node)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                tsi.sgns_o2(node, ctx, walks, seeds, w, n, packed, lr, 1.0, tsi.MODE_HOGWILD,
                            hot=hot, opts={"max_waves": mw} if mw else None)
                ev[1].record()
                torch.cuda.synchronize()
                loss = ti.compact_loss(node, ctx, ri, rp, rn)
                pt = {"hot": spec, "hot_rows": nhot, "max_waves": mw, "loss": loss,
                      "rel_to_seq": (loss - fx["seq_loss"]) / fx["seq_loss"],
                      "launch_ms": ev[0].elapsed_time(ev[1])}
                out["points"].append(pt)
                print(json.dumps(pt), flush=True)
                del node, ctx
                torch.cuda.empty_cache()
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
