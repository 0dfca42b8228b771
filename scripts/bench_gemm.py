#!/usr/bin/env python3
"""Decode-GEMM microbenchmark + autotuner: skinny HIP kernel vs F.linear (hipBLASLt).

Every variant is captured in a HIP graph of --iters calls (no host launch cost in
the number) with weights rotating through a pool larger than the 256 MiB Infinity
Cache, so each call streams its weights from HBM.  Variants are timed in
interleaved rounds in one process (guide §5.4 rule 24).

  Projections are timed together with what consumes them in the decode step (consumer_of):
  an o/down GEMM with its add + RMSNorm (which sums split-K slabs itself), a QKV GEMM without
  a reduce (attention sums its slabs) -- a separate reduce launch would bias the table against
  split-K.  --no-consumer times the bare op with its reduce.

  --tune  sweeps (cfg, split-K) per (M-tile bucket, N, K) and writes the winners to
          enterprise_inference_amd/ops/gemm_tuning.json (read by ops/gemm.py).  Several --m
          values in one 16-row bucket are scored together: the bucket's pick is the variant with
          the least summed time over those rows (e.g. --m 1 8 16 17 24 32 ...).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from enterprise_inference_amd.ops import gemm  # noqa: E402

SHAPES = {  # name: (N, K, swiglu)
    "qkv_8b": (6144, 4096, False), "o_8b": (4096, 4096, False),
    "gate_up_8b": (28672, 4096, True), "down_8b": (4096, 14336, False),
    # grid-fill probes: the 8B gate_up at 196 / 256 workgroups of 128 rows (224 in the model)
    "gate_up_8b_w196": (25088, 4096, True), "gate_up_8b_w256": (32768, 4096, True),
    "lm_head_8b": (128256, 4096, False),
    "qkv_70b_tp8": (1280, 8192, False), "o_70b_tp8": (8192, 1024, False),
    "gate_up_70b_tp8": (7168, 8192, True), "down_70b_tp8": (8192, 3584, False),
    "lm_head_70b_tp8": (16032, 8192, False),
    # Llama-3.3-70B on one GPU (profiles/sizing_70b_tp1_r1.md)
    "qkv_70b": (10240, 8192, False), "o_70b": (8192, 8192, False),
    "gate_up_70b": (57344, 8192, True), "down_70b": (8192, 28672, False),
    "lm_head_70b": (128256, 8192, False),
    # Llama-3.x-70B at TP4 (the reference's 70B deployment) and Llama-3.1-405B at TP8, per rank
    "qkv_70b_tp4": (2560, 8192, False), "o_70b_tp4": (8192, 2048, False),
    "gate_up_70b_tp4": (14336, 8192, True), "down_70b_tp4": (8192, 7168, False),
    "lm_head_70b_tp4": (32064, 8192, False),
    "qkv_405b_tp8": (2304, 16384, False), "o_405b_tp8": (16384, 2048, False),
    "gate_up_405b_tp8": (13312, 16384, True), "down_405b_tp8": (16384, 6656, False),
    "lm_head_405b_tp8": (16032, 16384, False),
    # Mistral-7B / Mixtral-8x7B LM heads (their attention projections are the 8B shapes)
    "lm_head_mistral": (32768, 4096, False), "lm_head_mixtral": (32000, 4096, False),
    # rest of the deployed catalog (reference core/playbooks/deploy-inference-models.yml):
    # Qwen2.5-32B (TP1, :909-977), DeepSeek-R1-Distill-Qwen-32B per TP2 rank (:1682-1768),
    # CodeLlama-34B (TP1, :1258-1340), Falcon3-7B (head_dim 256, :1342-1425)
    "qkv_qwen32b": (7168, 5120, False), "o_qwen32b": (5120, 5120, False),
    "gate_up_qwen32b": (55296, 5120, True), "down_qwen32b": (5120, 27648, False),
    "lm_head_qwen32b": (152064, 5120, False),
    "qkv_qwen32b_tp2": (3584, 5120, False), "o_qwen32b_tp2": (5120, 2560, False),
    "gate_up_qwen32b_tp2": (27648, 5120, True), "down_qwen32b_tp2": (5120, 13824, False),
    "lm_head_qwen32b_tp2": (76032, 5120, False),
    "qkv_codellama34b": (10240, 8192, False), "o_codellama34b": (8192, 8192, False),
    "gate_up_codellama34b": (44032, 8192, True), "down_codellama34b": (8192, 22016, False),
    "lm_head_codellama34b": (32000, 8192, False),
    "qkv_falcon3_7b": (5120, 3072, False), "o_falcon3_7b": (3072, 3072, False),
    "gate_up_falcon3_7b": (46080, 3072, True), "down_falcon3_7b": (3072, 23040, False),
    "lm_head_falcon3_7b": (131072, 3072, False),
    # Llama-4-Scout-17B-16E on one GPU (reference deploy-inference-models.yml:821-891): the
    # attention projections, the shared expert and the 202k-row LM head (routed experts run
    # the grouped MoE kernels)
    "qkv_scout": (7168, 5120, False), "o_scout": (5120, 5120, False),
    "shared_gate_up_scout": (16384, 5120, True), "shared_down_scout": (5120, 8192, False),
    "lm_head_scout": (202048, 5120, False),
    # Llama-3.2-3B (attention projections = the Falcon3-7B shapes), Qwen3-4B-Instruct-2507 and
    # Qwen3-1.7B (the reference serves these on Xeon, deploy-inference-models.yml; here on GPU)
    "gate_up_llama3b": (16384, 3072, True), "down_llama3b": (3072, 8192, False),
    "lm_head_llama3b": (128256, 3072, False),
    "qkv_qwen3_4b": (6144, 2560, False), "o_qwen3_4b": (2560, 4096, False),
    "gate_up_qwen3_4b": (19456, 2560, True), "down_qwen3_4b": (2560, 9728, False),
    "lm_head_qwen3_4b": (151936, 2560, False),
    "qkv_qwen3_1_7b": (4096, 2048, False), "o_qwen3_1_7b": (2048, 2048, False),
    "gate_up_qwen3_1_7b": (12288, 2048, True), "down_qwen3_1_7b": (2048, 6144, False),
    "lm_head_qwen3_1_7b": (151936, 2048, False),
    # gate_up grid-size probes (8B K): 196 / 224 (the real shape) / 256 four-pair workgroups
    "gu_probe_196": (25088, 4096, True), "gu_probe_256": (32768, 4096, True),
}


def consumer_of(name: str) -> str:
    """What consumes this projection's output in the decode step, so the tuner times the pair
    the engine runs instead of charging split-K variants a reduce launch the engine never makes:
      "norm"   o / down projections: the split-K slabs (or the bf16 tile) go straight into the
               residual add + RMSNorm kernel (splitk_add_rmsnorm / fused_add_rms_norm; at TP > 1
               the fused all-reduce kernel, which stages them the same way);
      "defer"  QKV: the slabs are summed in the decode attention's fused prologue (its cost per
               slab is small and paid by attention, not timed here) while they fit its LDS
               staging; a larger split is timed with the reduce launch the engine then runs;
      "plain"  everything else (LM head, SwiGLU): the op as the engine calls it."""
    if name.startswith(("o_", "down_", "shared_down")):
        return "norm"
    if name.startswith("qkv_"):
        return "defer"
    return "plain"


# q heads per KV head of each QKV shape: the decode attention stages the QKV split-K slabs of a
# (sequence, KV head) in LDS while sk * (G + 2) <= 68 (csrc/kernels/attention.hip); past that
# the engine reduces them in a launch of their own first (ops/attention.py), timed with the GEMM
QKV_GROUP = {"qkv_8b": 4, "qkv_70b_tp8": 8, "qkv_70b": 8, "qkv_70b_tp4": 8, "qkv_405b_tp8": 16,
             "qkv_qwen32b": 5, "qkv_qwen32b_tp2": 5, "qkv_codellama34b": 8,
             "qkv_falcon3_7b": 3, "qkv_scout": 5, "qkv_qwen3_4b": 4, "qkv_qwen3_1_7b": 2}


def qkv_max_sk(name: str) -> int:
    g = QKV_GROUP.get(name)
    return 68 // (g + 2) if g else 1 << 30


def graph_time(fn, iters, rounds=3):
    torch.cuda.synchronize()
    fn(0)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
        with torch.cuda.graph(g, stream=s):
            for i in range(iters):
                fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / iters * 1e3)
    del g
    return best   # us per call


def write_table(tuned, tuned_wg, out=None):
    table = {"device": torch.cuda.get_device_name(0), "entries": tuned, "wg_entries": tuned_wg}
    for path in [gemm.TUNING_FILE] + ([out] if out else []):
        with open(path, "w") as f:
            json.dump(table, f, indent=0, sort_keys=True)


def bucket_pick(b, margin=1.02):
    """A bucket's table entry from its summed timings: ``b`` = {"rows": [M...], "hip": summed
    hipBLASLt us, "var": {(cfg, sk): [summed us, rows timed]}}.  Only variants timed (valid,
    spill-free) at every row compete; [-1, 1] (hipBLASLt) unless the best skinny variant is
    within ``margin`` of it.  Returns (entry, best summed us, sorted [(us, (cfg, sk))])."""
    full = sorted((v[0], c) for c, v in b["var"].items() if v[1] == len(b["rows"]))
    if not full:
        return [-1, 1], b["hip"], full
    to, (cfg, sk) = full[0]
    return ([cfg, sk] if to < b["hip"] * margin else [-1, 1]), to, full


def candidates(M, N, K, swiglu):
    out = []
    for cfg in gemm.CFGS:
        nk = K // gemm.cfg_kc(cfg)
        for sk in range(1, nk + 1):
            if nk % sk or not gemm.valid(N, K, swiglu, cfg, sk, M=M):
                continue
            rows = gemm.cfg_rows(cfg) if not swiglu else gemm.cfg_rows(cfg)
            grid = (N // rows) * sk
            if sk > 1 and grid > 4096:
                continue
            if grid < 64 and sk < nk:
                continue
            out.append((cfg, sk))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[1, 16, 32, 48, 64, 80, 96, 112, 128])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--consumer", action=argparse.BooleanOptionalAction, default=True,
                    help="time each projection with its decode-step consumer (consumer_of): "
                         "o/down + add+RMSNorm, QKV with the slabs left to attention")
    ap.add_argument("--sweep", action="store_true", help="time every candidate (no table write)")
    ap.add_argument("--check", action="store_true",
                    help="sweep, and report the tuning table's pick against the best (regret) at "
                         "each M -- the table is timed at one M per 16-row bucket")
    ap.add_argument("--out", default=None, help="also write the tuning table here")
    ap.add_argument("--persist", action="store_true",
                    help="also copy the table into the PVC tuning cache ($EIA_CACHE_DIR)")
    ap.add_argument("--all", action="store_true", help="print every timed (cfg, sk) variant")
    ap.add_argument("--packed", action="store_true",
                    help="sweep the tile-packed-weight configurations (cfg bit 6)")
    ap.add_argument("--wgpack", action="store_true",
                    help="sweep the workgroup-packed forms (cfg bit 10) beside the plain ones")
    a = ap.parse_args()
    tuned, tuned_wg = {}, {}
    if a.tune and os.path.exists(gemm.TUNING_FILE):
        raw = json.load(open(gemm.TUNING_FILE))
        tuned, tuned_wg = raw.get("entries", {}), raw.get("wg_entries", {})
    for name in a.shapes:
        N, K, swiglu = SHAPES[name]
        wbytes = N * K * 2
        pool = max(2, int(600e6 // wbytes) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(pool)]
        wps = [gemm.pack_weight(w) for w in ws] if a.packed else ws
        wgp = {}    # waves -> workgroup-packed copies of the pool (cfg bit 10)

        def wg_pool(cfg):
            key = gemm.cfg_waves(cfg)
            if key not in wgp:
                wgp[key] = [gemm.pack_weight_wg(w, cfg, swiglu) for w in ws]
            return wgp[key]
        buckets = {}   # --tune: m-tile bucket -> summed times over its --m rows
        for M in a.m:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            if swiglu:
                I = N // 2
                base = lambda i: (lambda y: F.silu(y[:, :I]) * y[:, I:])(F.linear(x, ws[i % pool]))
            else:
                base = lambda i: F.linear(x, ws[i % pool])
            cons = consumer_of(name) if a.consumer else "plain"
            if cons == "norm":
                from enterprise_inference_amd.ops import norm as norm_ops
                res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) * 0.1
                wn = torch.ones(N, device="cuda", dtype=torch.bfloat16)
                base = lambda i: norm_ops.fused_add_rms_norm(F.linear(x, ws[i % pool]), res, wn,
                                                             1e-5)

                def skinny_call(i, cfg, sk, src):
                    y = gemm.skinny(x, src[i % pool], cfg=cfg, sk=sk, defer_reduce=True)
                    if isinstance(y, gemm.SplitK):
                        return gemm.splitk_add_rmsnorm(y, res, wn, 1e-5)
                    return norm_ops.fused_add_rms_norm(y, res, wn, 1e-5)
            elif cons == "defer":
                cap = qkv_max_sk(name)

                def skinny_call(i, cfg, sk, src):
                    # past the attention's staging capacity the engine reduces the slabs first
                    # (ops/attention.py decode_rope_attention): time that launch too
                    return gemm.skinny(x, src[i % pool], cfg=cfg, sk=sk,
                                       defer_reduce=sk <= cap)
            else:
                def skinny_call(i, cfg, sk, src):
                    return gemm.skinny(x, src[i % pool], cfg=cfg, sk=sk)
            tb = graph_time(base, a.iters)
            cands = candidates(M, N, K, swiglu) if (a.tune or a.sweep or a.check) else \
                [c for c in [gemm.choose(M, N, K, swiglu)] if c[0] >= 0]
            if a.packed:
                cands = [(c, sk) for c in gemm.PACKED_CFGS for sk in {s for _, s in cands}
                         if gemm.valid(N, K, swiglu, c, sk, M=M)
                         and (N // gemm.cfg_rows(c)) * sk <= 4096]
            if a.wgpack:
                # the table's plain pick against the workgroup-packed forms at every split
                # (--tune --wgpack: the plain entries stay, the packed picks go to wg_entries)
                pc, ps = gemm.choose(M, N, K, swiglu)
                cands = ([(pc, ps)] if pc >= 0 else []) + [
                    (c, sk) for c in gemm.WGPACK_CFGS for sk in (1, 2, 3, 4, 6, 8, 12, 16)
                    if gemm.valid(N, K, swiglu, c, sk, M=M)
                    and K % (sk * gemm.cfg_kc(c)) == 0 and (N // gemm.cfg_rows(c)) * sk <= 4096
                    and (N // gemm.cfg_rows(c)) * sk >= 64]
            if not cands:
                print(json.dumps({"shape": name, "M": M, "hipblaslt_us": round(tb, 2),
                                  "hipblaslt_TBps": round(wbytes / tb / 1e6, 2),
                                  "note": "tuned table routes this shape to hipBLASLt"}), flush=True)
                continue
            results = []
            for cfg, sk in cands:
                src = wg_pool(cfg) if cfg & 1024 else (wps if cfg & 64 else ws)
                if swiglu:
                    f = lambda i, cfg=cfg, sk=sk, src=src: gemm.swiglu_gemm(
                        x, src[i % pool], cfg=cfg, sk=sk)
                else:
                    f = lambda i, cfg=cfg, sk=sk, src=src: skinny_call(i, cfg, sk, src)
                results.append((graph_time(f, a.iters), cfg, sk))
            results.sort(key=lambda r_: r_[0])
            to, cfg, sk = results[0]
            r = {"shape": name, "M": M, "N": N, "K": K, "cfg": cfg, "sk": sk,
                 "ours_us": round(to, 2), "hipblaslt_us": round(tb, 2),
                 "ours_TBps": round(wbytes / to / 1e6, 2), "hipblaslt_TBps": round(wbytes / tb / 1e6, 2),
                 "speedup": round(tb / to, 2),
                 "runner_up": [(round(t, 1), c, s) for t, c, s in results[1:4]]}
            if a.all:
                r["all"] = [(round(t, 1), c, s) for t, c, s in results]
            if a.check:
                pick = gemm.choose(M, N, K, swiglu)
                tp = next((t for t, c, s_ in results if (c, s_) == tuple(pick)), None)
                if tp is None and pick[0] >= 0:   # table pick outside the candidate list
                    f = (lambda i: gemm.swiglu_gemm(x, ws[i % pool], cfg=pick[0], sk=pick[1])) \
                        if swiglu else \
                        (lambda i: skinny_call(i, pick[0], pick[1], ws))
                    tp = graph_time(f, a.iters)
                if pick[0] < 0:
                    tp = tb
                r["table_pick"] = list(pick)
                r["table_us"] = round(tp, 2)
                r["regret_pct"] = round(100.0 * (tp / min(to, tb) - 1.0), 1)
            print(json.dumps(r), flush=True)
            if a.tune:
                b = buckets.setdefault(gemm.m_bucket(M), {"rows": [], "hip": 0.0, "var": {}})
                b["rows"].append(M)
                b["hip"] += tb
                for t, c, s_ in results:
                    e = b["var"].setdefault((c, s_), [0.0, 0])
                    e[0] += t
                    e[1] += 1
        for mt, b in sorted(buckets.items()):
            key = f"{mt},{N},{K},{int(swiglu)}"
            if a.wgpack:
                # packed pick: the best packed variant timed at every row of the bucket, kept
                # when it beats the plain entry (timed in the same run) by >= 1 %
                full = sorted((v[0], c) for c, v in b["var"].items()
                              if v[1] == len(b["rows"]))
                plain = [(t, c) for t, c in full if not c[0] & 1024]
                packed = [(t, c) for t, c in full if c[0] & 1024]
                ref_t = plain[0][0] if plain else b["hip"]
                if packed and packed[0][0] < 0.99 * ref_t:
                    # third element: the gain in % of the plain time, which ranks the packed
                    # copies when the memory budget cannot hold them all (attach_wg_packed)
                    tuned_wg[key] = list(packed[0][1]) + [round(100.0 * (1 - packed[0][0] / ref_t), 1)]
                else:
                    tuned_wg.pop(key, None)
                print(json.dumps({"shape": name, "bucket": mt, "rows": b["rows"],
                                  "wg_pick": tuned_wg.get(key), "plain_sum_us": round(ref_t, 2),
                                  "wg_sum_us": round(packed[0][0], 2) if packed else None}),
                      flush=True)
                continue
            tuned[key], to, full = bucket_pick(b)
            print(json.dumps({"shape": name, "bucket": mt, "rows": b["rows"], "pick": tuned[key],
                              "sum_us": round(to, 2), "hipblaslt_sum_us": round(b["hip"], 2),
                              "runner_up": [(round(t, 1), c) for t, c in full[1:3]]}), flush=True)
        del ws, wps, wgp
        torch.cuda.empty_cache()
        if a.tune:
            write_table(tuned, tuned_wg, a.out)     # after every shape: a cut-off run keeps them
    if a.tune:
        print("wrote", gemm.TUNING_FILE)
        if a.persist:
            from enterprise_inference_amd.utils.cache_dir import persist
            print("persisted", persist(gemm.TUNING_FILE, "gemm_tuning.json"))


if __name__ == "__main__":
    main()
