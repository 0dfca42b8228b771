"""Deploy-layer placement and version-pin checks (no cluster, no helm binary).

1. Every infrastructure workload the operator CLI installs -- ingress-nginx, APISIX (gateway,
   etcd, ingress controller), Keycloak, Prometheus / Alertmanager / Grafana, istiod, LiteLLM
   and Langfuse -- is rendered from the values its playbook passes (Ansible's Jinja evaluated
   here against inventory/metadata/vars/inference_common.yml, charts through
   scripts/helm_lite.py), and its pod placement (nodeSelector, required node affinity,
   tolerations) is checked with the scheduler's node predicates against the two node layouts
   the deployment produces (core/playbooks/label-nodes.yml):

   * the north-star single node: 8x MI355X, control plane + worker, untainted, labelled
     role=inference (label-nodes.yml overwrites role=infra on a one-node cluster);
   * a multi-node infra control plane: role=infra, control-plane taint.

   Reference placement: affinity (role In [infra]) OR (control-plane Exists) plus the
   control-plane tolerations (/root/reference/core/helm-charts/apisix-helm/values.yaml:19-80,
   /root/reference/core/playbooks/deploy-ingress-controller.yml:76-95).

2. Every pin in inventory/metadata/inference-metadata.cfg reaches what installs it: passed
   by a component script as an --extra-vars name its playbook reads (chart pins in a
   `chart_version:`), or read directly by the shell (kubespray checkout, brownfield
   interpreter).  Also: every extra-var a component passes is read by its playbook, which is
   how the amd_gpu_operator / amd_gpu_operator_version miswire shipped.
"""

from __future__ import annotations

import glob
import json
import os
import re
import sys
import tempfile

import jinja2
import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORE = os.path.join(ROOT, "core")
PB = os.path.join(CORE, "playbooks")
CHARTS = os.path.join(CORE, "helm-charts")
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import helm_lite  # noqa: E402

CP = "node-role.kubernetes.io/control-plane"

NODES = {
    "single-node (role=inference, untainted control plane)": {
        "labels": {"role": "inference", "accelerator": "amd-mi355x", CP: ""},
        "taints": [],
    },
    "infra control plane (role=infra, tainted)": {
        "labels": {"role": "infra", CP: ""},
        "taints": [{"key": CP, "effect": "NoSchedule"}],
    },
}

# ------------------------------------------------------------------ scheduler predicates


def _expr_ok(expr: dict, labels: dict) -> bool:
    k, op, vals = expr["key"], expr["operator"], expr.get("values") or []
    if op == "In":
        return k in labels and labels[k] in vals
    if op == "NotIn":
        return k not in labels or labels[k] not in vals
    if op == "Exists":
        return k in labels
    if op == "DoesNotExist":
        return k not in labels
    raise AssertionError(f"operator {op}")


def _tolerated(taint: dict, tols: list) -> bool:
    for t in tols or []:
        if t.get("effect") and t["effect"] != taint["effect"]:
            continue
        if t.get("operator", "Equal") == "Exists":
            if not t.get("key") or t["key"] == taint["key"]:
                return True
        elif t.get("key") == taint["key"] and t.get("value") == taint.get("value"):
            return True
    return False


def schedulable(spec: dict, node: dict) -> bool:
    """NodeSelector + required node affinity + taint/toleration predicates of one pod spec."""
    labels = node["labels"]
    for k, v in (spec.get("nodeSelector") or {}).items():
        if labels.get(k) != v:
            return False
    na = ((spec.get("affinity") or {}).get("nodeAffinity") or {})
    req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
    if req:
        terms = req["nodeSelectorTerms"]
        if not any(all(_expr_ok(e, labels) for e in t.get("matchExpressions", []))
                   for t in terms):
            return False
    return all(_tolerated(t, spec.get("tolerations")) for t in node["taints"]
               if t["effect"] in ("NoSchedule", "NoExecute"))


def test_predicates_reject_the_old_selector():
    old = {"nodeSelector": {"role": "infra"}}
    assert not any(schedulable(old, n) for n in NODES.values())


# ------------------------------------------------------------------ Ansible value rendering


class _Undef(jinja2.ChainableUndefined):
    pass


def _env():
    env = jinja2.Environment(undefined=_Undef)
    env.filters["bool"] = lambda v: str(v).lower() in ("1", "true", "yes", "on")
    env.filters["to_json"] = lambda v: json.dumps(v)
    env.filters["from_yaml"] = yaml.safe_load
    return env


_FULL = re.compile(r"^\s*\{\{(.*)\}\}\s*$", re.S)


def _eval(obj, ctx, env):
    """Ansible-style templating: a string that is one {{ expr }} yields the object."""
    if isinstance(obj, dict):
        return {k: _eval(v, ctx, env) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_eval(v, ctx, env) for v in obj]
    if isinstance(obj, str) and "{{" in obj:
        m = _FULL.match(obj)
        if m and "{{" not in m.group(1):
            v = env.compile_expression(m.group(1).strip(), undefined_to_none=False)(**ctx)
            if isinstance(v, jinja2.Undefined):
                return ""
            return _eval(v, ctx, env) if isinstance(v, (str, dict, list)) else v
        return env.from_string(obj).render(**ctx)
    return obj


def _ctx(**extra):
    env = _env()
    raw = yaml.safe_load(open(os.path.join(CORE, "inventory/metadata/vars/inference_common.yml")))
    ctx = {"secret_name": "ai.example.com", "playbook_dir": PB, "platform": "vanilla",
           "kc_replicas": 1, "cert_file": "c", "key_file": "k"}
    ctx.update(extra)
    for _ in range(3):   # resolve vars that reference other vars
        ctx.update({k: _eval(v, {**ctx, **raw}, env) for k, v in raw.items()})
    return ctx, env


def _task(playbook: str, name: str) -> dict:
    plays = yaml.safe_load(open(os.path.join(PB, playbook)))
    for play in plays:
        for t in play.get("tasks", []):
            if t.get("name") == name:
                return t
    raise AssertionError(f"{playbook}: no task {name!r}")


def _helm_values(playbook: str, name: str, **extra) -> dict:
    ctx, env = _ctx(**extra)
    t = _task(playbook, name)
    h = t["kubernetes.core.helm"]
    vals: dict = {}
    for f in h.get("values_files", []):
        path = _eval(f, ctx, env)
        vals = _merge(vals, yaml.safe_load(open(path)))
    return _merge(vals, _eval(h.get("values") or {}, ctx, env))


def _merge(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in b.items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def _placement(d: dict) -> dict:
    return {k: d[k] for k in ("nodeSelector", "affinity", "tolerations") if k in d}


def _pod_spec_of(docs, kind="Deployment"):
    return [d["spec"]["template"]["spec"] for d in docs if d["kind"] == kind]


def _infra_workloads():
    out = {}
    ing = _helm_values("deploy-ingress-controller.yml", "ingress-nginx")
    out["ingress-nginx controller"] = _placement(ing["controller"])
    for plat in ("vanilla", "openshift"):
        ap = _helm_values("deploy-keycloak-tls-cert.yml", "APISIX", platform=plat)
        out[f"apisix gateway ({plat})"] = _placement(ap)
        out[f"apisix etcd ({plat})"] = _placement(ap["etcd"])
        out[f"apisix ingress-controller ({plat})"] = _placement(ap["ingress-controller"])
        assert ap["etcd"]["image"]["repository"] == "bitnamilegacy/etcd"
    kc = _helm_values("deploy-keycloak-tls-cert.yml", "Keycloak")
    out["keycloak"] = _placement(kc)
    obs = _helm_values("deploy-observability.yml", "kube-prometheus-stack",
                       grafana_admin_password="x")
    out["prometheus"] = _placement(obs["prometheus"]["prometheusSpec"])
    out["alertmanager"] = _placement(obs["alertmanager"]["alertmanagerSpec"])
    out["grafana"] = _placement(obs["grafana"])
    ist = _helm_values("deploy-istio.yml", "istiod (ambient profile)")
    out["istiod"] = _placement(ist["pilot"])
    # LiteLLM: the playbook's values rendered through the chart's own templates
    gw = _helm_values("deploy-genai-gateway.yml", "Gateway chart", litellm_master_key="m",
                      litellm_salt_key="s")
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
        yaml.safe_dump(gw, f)
    try:
        docs = helm_lite.render_chart(os.path.join(CHARTS, "genai-gateway"), [f.name], {},
                                      release="genai-gateway")
    finally:
        os.unlink(f.name)
    specs = _pod_spec_of(docs)
    assert specs, "genai-gateway rendered no Deployment"
    out["litellm"] = _placement(specs[0])
    # Langfuse: the trace values file is an Ansible template (lookup('template')); the
    # playbook merges the pod placement into it
    ctx, env = _ctx()
    src = open(os.path.join(CHARTS, "genai-gateway-trace/values.yaml")).read()
    tv = yaml.safe_load(env.from_string(src).render(**ctx))
    place = _task("deploy-genai-gateway.yml", "Trace pods on infra or control-plane nodes")
    tv = _merge(tv, _eval(place["vars"]["trace_placement"], ctx, env))
    out["langfuse web"] = _placement(tv["langfuse"]["web"])
    out["langfuse worker"] = _placement(tv["langfuse"]["worker"])
    return out


WORKLOADS = _infra_workloads()


@pytest.mark.parametrize("node", list(NODES))
@pytest.mark.parametrize("workload", sorted(WORKLOADS))
def test_infra_workload_schedules(workload, node):
    spec = WORKLOADS[workload]
    assert spec, f"{workload}: no placement rendered"
    assert schedulable(spec, NODES[node]), (workload, node, spec)


def test_infra_workloads_stay_off_plain_gpu_workers():
    """In a multi-node cluster the infra pods do not land on untainted GPU workers."""
    worker = {"labels": {"role": "inference", "accelerator": "amd-mi355x"}, "taints": []}
    for w, spec in WORKLOADS.items():
        assert not schedulable(spec, worker), w


def test_no_bare_infra_node_selector_left():
    for f in glob.glob(CORE + "/**/*.y*ml", recursive=True):
        txt = "\n".join(ln for ln in open(f).read().splitlines()
                        if not ln.lstrip().startswith("#"))
        assert not re.search(r"nodeSelector:\s*\{\s*['\"]?role['\"]?\s*:\s*['\"]?infra", txt), f
        assert "'role': 'infra'" not in txt, f


def test_model_pods_place_on_gpu_nodes_only():
    """vllm model pods (mi355x-values) run on the single node and stay off a tainted infra
    control plane."""
    docs = helm_lite.render_chart(os.path.join(CHARTS, "vllm"),
                                  [os.path.join(CHARTS, "vllm", "mi355x-values.yaml")],
                                  {"LLM_MODEL_ID": "meta-llama/Llama-3.1-8B-Instruct"},
                                  release="vllm-llama-8b")
    spec = _pod_spec_of(docs)[0]
    single, infra = NODES.values()
    assert schedulable(spec, single)
    assert not schedulable(spec, infra)


# ------------------------------------------------------------------ version pins


def _metadata():
    out = {}
    for line in open(os.path.join(CORE, "inventory/metadata/inference-metadata.cfg")):
        line = line.strip()
        if line and not line.startswith("#"):
            k, v = line.split("=", 1)
            out[k.strip()] = v.strip().strip('"')
    return out


def _playbook_text(path: str) -> str:
    """The playbook plus every task file under playbooks/tasks (include_tasks targets)."""
    txt = open(path).read()
    for f in glob.glob(os.path.join(PB, "tasks", "*.yml")):
        txt += open(f).read()
    return txt


def _invocations():
    """(script, playbook, {extra-var name: shell expression}) for every ansible-playbook call
    in core/lib whose extra-vars are given inline or via model_extra_vars."""
    model_vars = open(os.path.join(CORE, "lib/models/install-model.sh")).read()
    mv = dict(re.findall(r"(\w+)=(\$\{[^}]*\}|\$\(\S+)", model_vars.split("model_extra_vars()")[1]
                         .split("\n}")[0]))
    out = []
    for f in glob.glob(CORE + "/lib/**/*.sh", recursive=True):
        src = open(f).read()
        local = {k: v.strip('"') for k, v in re.findall(r'local (\w+)=("[^"]*"|\S+)', src)}
        for m in re.finditer(r"ansible-playbook((?:\\\n|[^\n])*)", src):
            call = m.group(1)
            for name, val in local.items():   # --extra-vars "${kc_vars}"
                call = call.replace("${" + name + "}", val).replace('"$' + name + '"', val)
            pb = re.search(r"playbooks/([\w.-]+\.yml)", call)
            if not pb:
                continue
            ev = dict(re.findall(r"(\w+)=(\$\{[^}]*\}|\$\(\S+)", call))
            if "$(model_extra_vars)" in call:
                ev.update(mv)
            out.append((os.path.relpath(f, CORE), pb.group(1), ev))
    return out


def test_every_metadata_pin_reaches_its_consumer():
    pins = _metadata()
    inv = _invocations()
    shell = "".join(open(f).read() for f in glob.glob(CORE + "/lib/**/*.sh", recursive=True))
    shell_direct = {"kubespray_version", "python3_interpreter"}
    for key in pins:
        if key in shell_direct:
            assert "${" + key in shell, key
            continue
        passed = [(s, pb, name) for s, pb, ev in inv for name, expr in ev.items()
                  if re.match(r"\$\{" + key + r"(:-[^}]*)?\}$", expr)]
        assert passed, f"{key}: no component passes it to a playbook"
        for s, pb, name in passed:
            txt = _playbook_text(os.path.join(PB, pb))
            assert re.search(r"\{\{[^}]*\b" + name + r"\b", txt), (key, s, pb, name)
            if "chart" in key or key in ("ingress_controller", "amd_gpu_operator"):
                assert re.search(r"chart_version:.*\b" + name + r"\b", txt), (key, pb, name)


def test_component_extra_vars_are_read():
    """Every extra-var name a component passes is read by the playbook it runs (the cluster
    context -- TLS files, platform names -- is handed to every playbook alike)."""
    broadcast = {"cert_file", "key_file", "gpu_platform", "kubernetes_platform", "secret_name"}
    unused = []
    for s, pb, ev in _invocations():
        path = os.path.join(PB, pb)
        if not os.path.exists(path):
            continue
        txt = _playbook_text(path)
        for name in set(ev) - broadcast:
            if not re.search(r"\b" + name + r"\b", txt):
                unused.append((s, pb, name))
    assert not unused, unused


def test_apisix_chart_pinned():
    assert _metadata()["apisix_chart_version"] == "2.8.1"
    h = _task("deploy-keycloak-tls-cert.yml", "APISIX")["kubernetes.core.helm"]
    assert "apisix_chart_version" in h["chart_version"]
    ing = _task("deploy-ingress-controller.yml", "ingress-nginx")["kubernetes.core.helm"]
    assert "ingress_controller" in ing["chart_version"]


def test_serving_values_match_bench():
    """The helm-deployed pods run what bench.py measures: no bucket-step override of the
    measured default (8), and the reference's 33024-token max model length."""
    vals = yaml.safe_load(open(os.path.join(CHARTS, "vllm", "mi355x-values.yaml")))
    for mid, cfg in vals["modelConfigs"].items():
        assert "VLLM_DECODE_BS_BUCKET_STEP" not in cfg.get("configMapValues", {}), mid
        args = cfg["extraCmdArgs"]
        assert args[args.index("--max-model-len") + 1] == "33024", mid


def test_ovms_token_in_secret():
    docs = helm_lite.render_chart(os.path.join(CHARTS, "ovms"), [], {"hfToken": "hf_abc"},
                                  release="ovms-qwen")
    dep = [d for d in docs if d["kind"] == "Deployment"][0]
    assert "hf_abc" not in json.dumps(dep)
    sec = [d for d in docs if d["kind"] == "Secret"]
    assert sec and sec[0]["stringData"]["HF_TOKEN"] == "hf_abc"
    env = dep["spec"]["template"]["spec"]["initContainers"][0]["env"]
    assert env[0]["valueFrom"]["secretKeyRef"]["name"] == "ovms-qwen-hf-token"
