"""Tier C at C5's kernel shape (tests/tierc_inputs.py C5: d = 256, n = 10, 1M-node graph, one
131,072-walk launch) as a function of the wavefronts in flight (come_launch_opts.max_waves):
held-out loss of the GPU Hogwild launch against the sequential oracle's (tests/golden/
tierc_c5_seq.json) and the launch time, to separate the concurrency effect from the kernel.

    python scripts/tierc_c5_waves.py [--waves 0,4096,2048,1024,512] [--out ...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", default="0,4096,2048,1024,512")
    ap.add_argument("--hot-p", default="")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    from tierc_inputs import C5_HYPER, c5_inputs, sgns_loss
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "tierc_c5_seq.json")))
    x = c5_inputs()
    assert x.digest == fx["inputs_sha256"]
    w, n, lr = C5_HYPER["window"], C5_HYPER["negative"], C5_HYPER["lr"]
    ri, rp, rn = x.heldout(w, n)
    dev = torch.device("cuda", 0)
    tab = torch.from_numpy(x.table.view(np.int32)).to(dev)
    packed = tsi.pack_table(tab)
    walks = torch.from_numpy(x.train).to(dev)
    seeds = torch.from_numpy(x.seeds.view(np.int64)).to(dev)
    out = {"seq_loss": fx["seq_loss"], "init_loss": fx["init_loss"], "points": []}
    shares = [float(v) for v in args.hot_p.split(",")] if args.hot_p else [tsi.DEFAULT_HOT_P]
    for share in shares:
        hot = tsi.hot_rows(tab, x.g.V, max(1, int(share * len(x.table))))
        for mw in [int(v) for v in args.waves.split(",")]:
            node = torch.from_numpy(x.node0).to(dev)
            ctx = torch.zeros_like(node)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            tsi.sgns_o2(node, ctx, walks, seeds, w, n, packed, lr, 1.0, tsi.MODE_HOGWILD,
                        hot=hot, opts={"max_waves": mw} if mw else None)
            ev[1].record()
            torch.cuda.synchronize()
            loss = sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), ri, rp, rn)
            pt = {"hot_share": share, "max_waves": mw, "loss": loss,
                  "rel_to_seq": (loss - fx["seq_loss"]) / fx["seq_loss"],
                  "launch_ms": ev[0].elapsed_time(ev[1])}
            out["points"].append(pt)
            print(json.dumps(pt), flush=True)
            del node, ctx
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
