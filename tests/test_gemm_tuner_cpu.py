"""scripts/bench_gemm.py bucket scoring (round 4): a 16-row bucket's table entry is the variant
with the least summed time over the bucket's timed rows, among variants timed at all of them;
hipBLASLt ([-1, 1]) wins unless the best skinny variant is within 2 %."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location("bench_gemm",
                                                  os.path.join(ROOT, "scripts", "bench_gemm.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bucket_pick_sums_rows_and_skips_partial_variants():
    bp = _mod().bucket_pick
    b = {"rows": [49, 56, 64], "hip": 150.0,
         "var": {(3, 8): [140.0, 3],        # best over all three rows
                 (2, 2): [90.0, 2],         # fastest sum but spills at one row: not eligible
                 (22, 8): [141.0, 3]}}
    entry, to, full = bp(b)
    assert entry == [3, 8] and to == 140.0
    assert [c for _, c in full] == [(3, 8), (22, 8)]


def test_bucket_pick_routes_to_hipblaslt():
    bp = _mod().bucket_pick
    b = {"rows": [17, 24, 32], "hip": 100.0, "var": {(24, 1): [103.0, 3]}}
    assert bp(b)[0] == [-1, 1]
    b["var"][(24, 1)][0] = 101.0                  # within the 2 % margin: keep the skinny kernel
    assert bp(b)[0] == [24, 1]
    assert bp({"rows": [1], "hip": 5.0, "var": {}})[0] == [-1, 1]


def test_wg_packed_selection(monkeypatch):
    """A weight that carries a workgroup-packed copy takes the table's packed pick for its
    batch bucket; without the copy (or without a packed pick) the plain entry stands."""
    import torch
    from enterprise_inference_amd.ops import gemm
    N, K = 4096, 4096
    monkeypatch.setattr(gemm, "_TUNED_WG", {(5, N, K, False): (1024 + 17, 4),
                                            (2, N, K, False): (1024 + 19, 4)})
    w = torch.nn.Parameter(torch.zeros(N, K, dtype=torch.bfloat16), requires_grad=False)
    assert gemm.choose_packed(65, N, K, False, w) is None           # no packed copy attached
    assert gemm.wg_layouts(N, K, False) == [2, 4]
    assert gemm.wg_layouts(N, K, False, max_m=32) == [4]            # buckets <= 2 only
    packed = torch.ones(N, K, dtype=torch.bfloat16)
    w.__dict__["_eia_wg"] = {(2, False): packed}
    cfg, sk, wp = gemm.choose_packed(65, N, K, False, w)
    assert (cfg, sk) == (1024 + 17, 4) and wp is packed
    assert gemm.choose_packed(20, N, K, False, w) is None            # layout 4 not attached
    assert gemm.choose_packed(5, N, K, False, w) is None             # bucket 1: no packed pick


def test_every_catalog_decode_shape_has_all_batch_buckets():
    """Every decode GEMM shape the tuner knows (the catalog's models, TP ranks included) has a
    table entry at each 16-row bucket up to 128 rows: a missing bucket would silently fall back
    to hipBLASLt at that batch size (1-3 TB/s there, profiles/gemm_tune_tp8_all_buckets_r6.log)."""
    import json
    bg = _mod()
    with open(os.path.join(ROOT, "enterprise_inference_amd", "ops", "gemm_tuning.json")) as f:
        table = json.load(f)["entries"]
    gaps = {}
    for name, (N, K, sw) in bg.SHAPES.items():
        if "probe" in name or name.startswith("gate_up_8b_w"):
            continue
        have = {int(k.split(",")[0]) for k in table if k.split(",", 1)[1] == f"{N},{K},{int(sw)}"}
        miss = [m for m in range(1, 9) if m not in have]
        if miss:
            gaps[name] = miss
    assert not gaps, gaps
