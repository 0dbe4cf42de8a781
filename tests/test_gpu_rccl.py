"""RCCL on the GPU: the multi-GPU exchange's collectives, stream waits and flag
all-reduces run through a real "nccl" (= RCCL) process group before the driver's first 8-GPU job.

A one-GPU box cannot hold two RCCL ranks on one device ("Duplicate GPU detected"), so the group has
ONE rank on cuda:0 and the exchanges are built with ``force_exchange=True`` (the test-only switch
that keeps them from short-circuiting world == 1).  Every collective the trainers issue then runs
as an RCCL kernel: the broadcast of the starting tables, the fp32 SUM all-reduce of the deltas in
buckets, the uint8 SUM all-reduce of touched_mean's per-row change counts, the uint8 MAX of the
row-sparse union and pick's priorities -- overlapped with live O2 Hogwild launches on the same
tables (start() before a launch, finish() after it), as Context2Vec(distributed=True) runs them.

With one rank every combine is the identity on the delta, so the arithmetic is known bit for bit:
after start() at tables W0 (sync base S0) and a launch that moves W0 to W1,
    S' = fp32(S0 + fp32(W0 - S0))     W' = W1 exactly (sum_r D_r - D_own == +0)
which distributed.reference_delta_sum / reference_touched_mean state in float64 (checked too).
"""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, out, combine, sparse):
    import torch
    import torch.distributed as dist
    res = {"ok": False}
    try:
        import come_amd.training_sdg_inner as tsi
        from come_amd.distributed import (DeltaAllReduce, SparseDeltaAllReduce,
                                          reference_delta_sum, reference_touched_mean)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0,
                                world_size=1)
        res["backend"] = dist.get_backend()
        g = torch.Generator(device="cpu").manual_seed(7)
        V, d, P, L, T = 50_000, 128, 4096, 40, 1_000_000
        node = ((torch.rand(V, d, generator=g) - 0.5) / d).to(dev)
        ctx = torch.zeros(V, d, device=dev)
        table = torch.randint(0, V, (T,), generator=g, dtype=torch.int32).to(dev)
        walks = [torch.randint(0, V, (P, L), generator=g, dtype=torch.int32).to(dev)
                 for _ in range(4)]
        seeds = [torch.randint(0, 2 ** 48, (P,), generator=g, dtype=torch.int64).to(dev)
                 for _ in range(4)]

        def launch(b):
            tsi.sgns_o2(node, ctx, walks[b], seeds[b], 5, 5, table, 0.1, 1.0, tsi.MODE_HOGWILD)

        cls = SparseDeltaAllReduce if sparse else DeltaAllReduce
        ex = cls([node, ctx], combine=combine, force_exchange=True, bucket_elems=1 << 20)
        checks = []
        launch(0)
        for b in (1, 2):
            w0 = [node.clone(), ctx.clone()]
            s0 = [s.clone() for s in ex.snap]
            ex.start()        # RCCL all-reduces on their own stream ...
            launch(b)         # ... beside an O2 launch on the same tables
            w1 = [node.clone(), ctx.clone()]
            ex.finish()
            torch.cuda.synchronize()
            for i, t in enumerate((node, ctx)):
                W0, S0 = w0[i].cpu().numpy(), s0[i].cpu().numpy()
                S = ex.snap[i].cpu().numpy()
                exp = (S0 + (W0 - S0).astype(np.float32)).astype(np.float32)
                ref = (reference_touched_mean(S0, [W0]) if combine == "touched_mean"
                       else reference_delta_sum(S0, [W0]))
                changed = int((W0.view(np.int32) != S0.view(np.int32)).any(axis=1).sum())
                checks.append({
                    "batch": b, "table": i, "rows_changed": changed,
                    "sync_bitexact": bool(np.array_equal(S.view(np.int32),
                                                         exp.view(np.int32))),
                    "sync_vs_ref_maxabs": float(np.abs(S.astype(np.float64) - ref).max()),
                    "table_bitexact": bool(torch.equal(t, w1[i])),
                    "launch_moved": bool(not torch.equal(w1[i], w0[i])),
                })
        ex.sync()             # the blocking exchange train() ends with
        torch.cuda.synchronize()
        res["final_equal"] = all(bool(torch.equal(t, s)) for t, s in zip((node, ctx), ex.snap))
        if not sparse:        # pick's uint8 MAX priorities through RCCL, blocking
            pk = DeltaAllReduce([node, ctx], combine="pick", force_exchange=True)
            before = [node.clone(), ctx.clone()]
            launch(3)
            moved = [node.clone(), ctx.clone()]
            pk.sync()
            torch.cuda.synchronize()
            res["pick_equal"] = all(
                bool(torch.equal(s, (b + (m - b)))) for s, b, m in zip(pk.snap, before, moved))
        res["checks"] = checks
        res["ok"] = True
        dist.destroy_process_group()
    except Exception as e:  # reported to the parent
        import traceback
        res["error"] = "%s\n%s" % (e, traceback.format_exc())
    with open(out, "w") as f:
        json.dump(res, f)


@pytest.mark.parametrize("combine,sparse", [("touched_mean", False), ("sum", False),
                                            ("touched_mean", True)])
def test_rccl_exchange_beside_live_o2_launches(tmp_path, combine, sparse):
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.json")
    p = mp.get_context("spawn").Process(target=_worker, args=(_free_port(), out, combine, sparse))
    p.start()
    p.join(100)
    if p.is_alive():
        p.kill()
        p.join(10)
        pytest.fail("RCCL worker did not finish within 100 s")
    assert p.exitcode == 0, p.exitcode
    res = json.load(open(out))
    assert res["ok"], res.get("error")
    assert res["backend"] == "nccl"
    print(json.dumps(res["checks"]))
    for c in res["checks"]:
        assert c["launch_moved"] and c["rows_changed"] > 0, c
        assert c["sync_bitexact"], c        # W_sync += the all-reduced delta, bit for bit
        assert c["table_bitexact"], c       # the overlapped launch's progress kept exactly
        assert c["sync_vs_ref_maxabs"] <= 1e-6, c
    assert res["final_equal"]
    if not sparse:
        assert res["pick_equal"]
