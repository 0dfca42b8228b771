#!/usr/bin/env python3
"""Run every row of the reference sizing guide on this box and tabulate ours vs Gaudi 3.

The reference publishes one performance table per model
(reference third_party/IBM/docs/sizing-guide.md:56-63 for Llama-3.1-8B on 1 Gaudi 3,
:69-76 for Llama-3.3-70B on 4 Gaudi 3): throughput (output tokens/s) and TTFT p90 for
eight "use cases" (input/output lengths) at the concurrency the guide calls the sweet spot.
Each row here is one `bench.py` child process at the same input/output lengths and the same
number of concurrent users (all arriving at once, ignore_eos, random-init weights,
synthetic prompts), so the comparison is per replica at equal load.

    python scripts/sizing_sweep.py --model 8b --out gpurun_out/sizing_8b.md
    python scripts/sizing_sweep.py --model 70b --cases chatbot describe

Every child runs under its own time limit; the first failure ends the sweep.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (use case, input, output, users, Gaudi-3 tok/s, Gaudi-3 TTFT p90 ms)
SIZING = {
    "8b": ("meta-llama/Llama-3.1-8B-Instruct", 1, [       # sizing-guide.md:56-63
        ("chatbot", 128, 128, 65, 3264, 1300),
        ("content_creation", 128, 2048, 35, 3172, 394),
        ("code_generation", 128, 4096, 35, 2799, 474),
        ("describe", 2048, 128, 210, 1318, 19463),
        ("suggest", 4096, 128, 135, 800, 18745),
        ("summarize", 8192, 128, 65, 391, 18412),
        ("translate", 1024, 1024, 65, 2854, 11815),
        ("correct", 2048, 2048, 35, 2463, 1921),
    ]),
    "70b": ("meta-llama/Llama-3.3-70B-Instruct", 4, [     # sizing-guide.md:69-76
        ("chatbot", 128, 128, 35, 1120, 613),
        ("content_creation", 128, 2048, 35, 1269, 586),
        ("code_generation", 128, 4096, 35, 1254, 605),
        ("describe", 2048, 128, 65, 486, 13348),
        ("suggest", 4096, 128, 40, 306, 18123),
        ("summarize", 8192, 128, 30, 161, 19952),
        ("translate", 1024, 1024, 35, 1158, 3320),
        ("correct", 2048, 2048, 60, 1060, 7589),
    ]),
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=sorted(SIZING), default="8b")
    ap.add_argument("--cases", nargs="*", default=None)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--timeout", type=int, default=420)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    model, ref_gpus, rows = SIZING[args.model]
    if args.cases:
        rows = [r for r in rows if r[0] in args.cases]
    lines = [f"### Sizing-guide sweep: {model}, TP={args.tp} on {args.tp}x MI355X "
             f"(reference: {ref_gpus}x Gaudi 3)", "",
             "| use case | in/out | users | ours tok/s | Gaudi 3 tok/s | ratio | ratio per card "
             "| ours TTFT p90 ms | Gaudi 3 TTFT p90 ms | TPOT p50 ms |",
             "|---|---|---:|---:|---:|---:|---:|---:|---:|---:|"]
    results = []
    for name, inp, outp, users, ref_tps, ref_ttft in rows:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", model,
               "--users", str(users), "--input-len", str(inp), "--output-len", str(outp),
               "--steps", str(args.steps), "--warmup", str(args.warmup),
               "--max-num-seqs", str(max(256, users)),
               "--max-num-batched-tokens", str(max(8192, inp)),
               # burst rounds only: a closed-loop window would wait out whole long-output requests
               "--closed-loop-s", "0"]
        if args.tp > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={args.tp}", "--master-addr", "127.0.0.1",
                   "--master-port", "29533"] + cmd[1:] + ["--tp", str(args.tp),
                                                           "--gpus", str(args.tp)]
        print(f"== {name}: {' '.join(cmd)}", flush=True)
        # the child's output goes to files; a heartbeat line a minute keeps a long row (a 4096-
        # token generation at 70B takes minutes) visibly alive to whatever watches this process
        import tempfile
        import time
        with tempfile.TemporaryFile("w+") as out, tempfile.TemporaryFile("w+") as err:
            p = subprocess.Popen(cmd, stdout=out, stderr=err, text=True)
            t0 = time.time()
            while True:
                try:
                    rc = p.wait(timeout=60)
                    break
                except subprocess.TimeoutExpired:
                    if time.time() - t0 > args.timeout:
                        p.kill()
                        p.wait()
                        rc = -9
                        break
                    print(f"   {name}: {time.time() - t0:.0f} s", flush=True)
            out.seek(0)
            err.seek(0)
            stdout, stderr = out.read(), err.read()
        if rc != 0:
            print(stdout[-2000:], stderr[-4000:], flush=True)
            print(f"{name} rc={rc}", flush=True)
            return rc if rc > 0 else 1
        js = [json.loads(ln) for ln in stdout.splitlines() if ln.startswith("{")]
        r = js[-1]
        results.append({"case": name, **r})
        ratio = r["value"] / ref_tps
        per_card = ratio * ref_gpus / args.tp
        lines.append(f"| {name} | {inp}/{outp} | {users} | {r['value']:.0f} | {ref_tps} | "
                     f"{ratio:.2f}x | {per_card:.2f}x | {r['ttft_p90_ms']:.0f} | {ref_ttft} | "
                     f"{r['tpot_p50_ms']:.2f} |")
        print(lines[-1], flush=True)
    text = "\n".join(lines) + "\n"
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)
        with open(os.path.splitext(args.out)[0] + ".jsonl", "w") as f:
            for r in results:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
