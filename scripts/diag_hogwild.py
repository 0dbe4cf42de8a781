"""Diagnostic: ComE end-to-end NMI vs Hogwild concurrency (come_set_option rows_per_wave)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "scripts"))
import come_e2e
from come_amd import _lib
cases = [dict(blocks=8, block_size=250, p_in=0.04, p_out=0.002, dim=64, walk_length=30,
              num_walks=4, n_init=3, seed=3),
         dict(blocks=50, block_size=2000, p_in=0.008, p_out=4e-5, dim=128, walk_length=40,
              num_walks=5, n_init=2, seed=3)]
for c in cases:
    for det in (True,):
        out = come_e2e.run(**c, deterministic=True, log=lambda s: None) if c["blocks"] == 8 else None
        if out:
            print(json.dumps({"V": c["blocks"] * c["block_size"], "mode": "sequential", "nmi": out["nmi"], "t": out["timings_s"]}), flush=True)
    for rpw in (0, 4096, 1024, 256, 64, 16):
        _lib.set_option("rows_per_wave", rpw)
        out = come_e2e.run(**c, log=lambda s: None)
        print(json.dumps({"V": c["blocks"] * c["block_size"], "rows_per_wave": rpw, "nmi": out["nmi"],
                          "t": out["timings_s"]}), flush=True)
    _lib.set_option("rows_per_wave", 0)
