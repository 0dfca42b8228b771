#!/usr/bin/env python3
"""Generate ibm_catalog.json (IBM Cloud deployable-architecture manifest) from the patterns.

The manifest lists one flavor per Terraform pattern (quickstart: existing VPC; standard: new
VPC) and one configuration entry per `variable` block of that pattern's variables.tf, so the
catalog can never drift from the Terraform inputs (tests/test_deploy_cpu.py checks it).
Parity: reference ibm_catalog.json (products[0].flavors[quickstart|standard].configuration).

    python scripts/gen_ibm_catalog.py            # rewrite ibm_catalog.json
    python scripts/gen_ibm_catalog.py --check    # exit 1 if the file is stale
"""

from __future__ import annotations

import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATTERNS = os.path.join(ROOT, "third_party", "IBM", "patterns")
OUT = os.path.join(ROOT, "ibm_catalog.json")

FLAVORS = [
    ("quickstart", "QuickStart", "Deploy into an existing VPC, subnet and security group: "
     "one 8-GPU AMD Instinct instance (single-node) or control-plane + GPU workers."),
    ("standard", "Standard", "Create a new VPC, security group, public gateway and subnet, "
     "then a multi-node cluster: CPU control-plane nodes plus 8-GPU AMD Instinct workers."),
]


def parse_variables(path: str):
    """Minimal HCL reader for `variable "x" { description/type/default/sensitive }` blocks."""
    text = open(path).read()
    out = []
    for m in re.finditer(r'variable\s+"(\w+)"\s*\{', text):
        depth, i = 1, m.end()
        while depth and i < len(text):
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        body = text[m.end():i - 1]
        desc = re.search(r'description\s*=\s*"([^"]*)"', body)
        typ = re.search(r'^\s*type\s*=\s*(\w+)', body, re.M)
        dflt = re.search(r'^\s*default\s*=\s*("([^"]*)"|[\w.]+)', body, re.M)
        sens = re.search(r'sensitive\s*=\s*true', body)
        item = {"key": m.group(1), "type": typ.group(1) if typ else "string",
                "description": desc.group(1) if desc else "",
                "required": dflt is None}
        if dflt is not None:
            raw = dflt.group(2) if dflt.group(2) is not None else dflt.group(1)
            if item["type"] == "number":
                raw = float(raw) if "." in raw else int(raw)
            elif raw in ("true", "false"):
                raw = raw == "true"
            elif raw == "null":
                raw = None
            item["default_value"] = raw
        if sens:
            item["type"] = "password"
        out.append(item)
    return out


def build() -> dict:
    flavors = []
    for i, (name, label, desc) in enumerate(FLAVORS, 1):
        flavors.append({
            "label": label, "name": name, "index": i, "install_type": "fullstack",
            "working_directory": f"third_party/IBM/patterns/{name}",
            "architecture": {"descriptions": desc, "features": [
                {"title": "AMD Instinct MI355X serving", "description":
                 "One serving pod per GPU (TP=1 for 8B-32B), TP=8 for 70B/405B, RCCL over xGMI."},
                {"title": "Gateway", "description":
                 "Keycloak + APISIX or LiteLLM GenAI gateway with Langfuse traces."}]},
            "configuration": parse_variables(os.path.join(PATTERNS, name, "variables.tf")),
        })
    return {"products": [{
        "label": "Enterprise Inference on AMD Instinct",
        "name": "da-enterprise-inference-amd",
        "product_kind": "solution",
        "tags": ["ai", "inference", "amd-instinct"],
        "keywords": ["LLM", "vLLM-compatible", "MI355X"],
        "short_description": "Provision IBM Cloud VPC instances with AMD Instinct GPUs and deploy "
                             "the Enterprise Inference stack (Kubernetes, gateway, models).",
        "offering_docs_url": "docs/getting-started.md",
        "flavors": flavors,
    }]}


def main() -> int:
    text = json.dumps(build(), indent=2) + "\n"
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        if cur != text:
            print("ibm_catalog.json is stale: run scripts/gen_ibm_catalog.py", file=sys.stderr)
            return 1
        return 0
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
