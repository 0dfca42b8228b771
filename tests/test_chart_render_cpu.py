"""Helm charts rendered per cluster platform (scripts/helm_lite.py: the Go-template subset the
charts use, no helm binary needed).  kubernetes_platform selects how a model, an embedding /
rerank service and the Keycloak /token endpoint are exposed -- the reference swaps template
files for the same effect (core/playbooks/deploy-inference-models.yml:85-258):

  vanilla   -> NGINX Ingress (class nginx)
  eks       -> ALB Ingress (class alb, shared group eks-genai)
  openshift -> Route (edge TLS)
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHARTS = os.path.join(ROOT, "core", "helm-charts")
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import helm_lite  # noqa: E402

EXPECT = {"vanilla": ("Ingress", "nginx"), "eks": ("Ingress", "alb"), "openshift": ("Route", None)}


def _exposure(docs):
    return [d for d in docs if d["kind"] in ("Ingress", "Route")]


def _render(chart, platform, apisix=False, files=(), extra=None):
    sets = {"platform": platform, "ingress.enabled": "true", "ingress.host": "ai.example.com",
            "ingress.secretname": "ai.example.com", "apisix.enabled": str(apisix).lower()}
    sets.update(extra or {})
    return helm_lite.render_chart(os.path.join(CHARTS, chart),
                                  [os.path.join(CHARTS, chart, f) for f in files], sets,
                                  release=f"{chart}-llama-8b")


@pytest.mark.parametrize("platform", ["vanilla", "eks", "openshift"])
@pytest.mark.parametrize("apisix", [False, True])
@pytest.mark.parametrize("chart,files,prefix", [
    ("vllm", ["mi355x-values.yaml"], "Llama-3.1-8B-Instruct"),
    ("tei", ["mi355x-values.yaml"], "bge-base-en-v1.5"),
    ("teirerank", ["mi355x-values.yaml"], "bge-reranker-base")])
def test_model_exposure_per_platform(chart, files, prefix, platform, apisix):
    docs = _render(chart, platform, apisix, files)
    exp = _exposure(docs)
    kind, cls = EXPECT[platform]
    assert [d["kind"] for d in exp] == [kind], [d["_template"] for d in exp]
    obj = exp[0]
    assert obj["metadata"].get("namespace", "default") == ("auth-apisix" if apisix else "default")
    backend_svc = "auth-apisix-gateway" if apisix else f"{chart}-llama-8b-service"
    if kind == "Route":
        spec = obj["spec"]
        assert spec["host"] == "ai.example.com" and spec["path"] == f"/{prefix}"
        assert spec["to"]["name"] == backend_svc
        assert spec["tls"]["termination"] == "edge"
        ann = obj["metadata"].get("annotations") or {}
        # without APISIX the router strips the model prefix itself
        assert ("haproxy.router.openshift.io/rewrite-target" in ann) == (not apisix)
    else:
        spec = obj["spec"]
        assert spec["ingressClassName"] == cls
        path = spec["rules"][0]["http"]["paths"][0]
        assert path["backend"]["service"]["name"] == backend_svc
        if cls == "alb":
            ann = obj["metadata"]["annotations"]
            assert ann["alb.ingress.kubernetes.io/group.name"] == "eks-genai"
            assert path["path"] == f"/{prefix}" and path["pathType"] == "Prefix"


def test_no_exposure_when_disabled():
    for platform in EXPECT:
        docs = helm_lite.render_chart(os.path.join(CHARTS, "vllm"),
                                      [os.path.join(CHARTS, "vllm", "mi355x-values.yaml")],
                                      {"platform": platform})
        assert not _exposure(docs)


def test_eks_without_apisix_strips_prefix_in_the_server():
    """An ALB cannot rewrite paths: the server gets --root-path /<model> (vLLM flag) and the
    TEI pods ROOT_PATH, only on EKS without the APISIX gateway."""
    def args(platform, apisix):
        dep = [d for d in _render("vllm", platform, apisix, ["mi355x-values.yaml"])
               if d["kind"] == "Deployment"][0]
        return dep["spec"]["template"]["spec"]["containers"][0]["args"]

    a = args("eks", False)
    assert a[a.index("--root-path") + 1] == "/Llama-3.1-8B-Instruct"
    assert "--root-path" not in args("eks", True)
    assert "--root-path" not in args("vanilla", False)
    dep = [d for d in _render("tei", "eks", False, ["mi355x-values.yaml"])
           if d["kind"] == "Deployment"][0]
    env = {e["name"]: e.get("value") for e in dep["spec"]["template"]["spec"]["containers"][0]["env"]}
    assert env["ROOT_PATH"] == "/bge-base-en-v1.5"


@pytest.mark.parametrize("platform", ["vanilla", "eks", "openshift"])
def test_keycloak_token_exposure(platform):
    docs = helm_lite.render_chart(os.path.join(CHARTS, "keycloak"), (),
                                  {"platform": platform, "host": "ai.example.com",
                                   "secretname": "ai.example.com"})
    kinds = sorted(d["kind"] for d in docs)
    assert "ApisixRoute" in kinds and "ApisixUpstream" in kinds
    exp = _exposure(docs)
    kind, cls = EXPECT[platform]
    token = [d for d in exp if "token" in d["metadata"]["name"]]
    assert len(token) == 1 and token[0]["kind"] == kind
    if kind == "Ingress":
        assert token[0]["spec"]["ingressClassName"] == cls
        assert token[0]["spec"]["rules"][0]["http"]["paths"][0]["path"] == "/token"
    else:
        assert token[0]["spec"]["path"] == "/token"
        # the Keycloak console gets its own Route on OpenShift
        assert any(d["metadata"]["name"] == "keycloak" for d in exp)


def test_deploy_model_task_passes_platform():
    import yaml
    tasks = yaml.safe_load(open(os.path.join(ROOT, "core/playbooks/tasks/deploy-model.yml")))
    helm = [t for t in tasks if "helm upgrade --install" in t["name"]][0]
    cmd = helm["ansible.builtin.command"]
    assert "--set platform={{ kubernetes_platform | default('vanilla') }}" in cmd


def test_root_path_middleware():
    from fastapi import FastAPI
    from fastapi.testclient import TestClient

    from enterprise_inference_amd.entrypoints.openai.api_server import _BearerAuth, _StripPrefix
    app = FastAPI()

    @app.get("/v1/models")
    def models():
        return {"ok": True}

    @app.get("/health")
    def health():
        return {}

    app.add_middleware(_BearerAuth, api_key="k")
    app.add_middleware(_StripPrefix, prefix="/Llama-3.1-8B-Instruct")
    c = TestClient(app)
    assert c.get("/Llama-3.1-8B-Instruct/v1/models").status_code == 401   # auth still applies
    assert c.get("/Llama-3.1-8B-Instruct/v1/models",
                 headers={"Authorization": "Bearer k"}).json() == {"ok": True}
    assert c.get("/health").status_code == 200


# ----------------------------------------------------------------------------- logs stack

def _deep_merge(a, b):
    out = dict(a)
    for k, v in b.items():
        out[k] = _deep_merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) \
            else v
    return out


@pytest.mark.parametrize("overlay", [None, "aws-s3-values.yaml"])
def test_logs_stack_values(overlay):
    """Loki SimpleScalable on an object store (MinIO by default, AWS S3 with the overlay), 7-day
    retention enforced by the compactor, OTLP resource attributes as index labels, the
    collector's PodMonitor and the tenant header on both the write and the read side."""
    import yaml
    base = os.path.join(CHARTS, "observability", "logs-stack")
    v = yaml.safe_load(open(os.path.join(base, "values.yaml")))
    if overlay:
        v = _deep_merge(v, yaml.safe_load(open(os.path.join(base, overlay))))
    loki = v["loki"]
    assert loki["deploymentMode"] == "SimpleScalable" and loki["fullnameOverride"] == "loki"
    assert loki["write"]["replicas"] == loki["loki"]["commonConfig"]["replication_factor"]
    assert loki["minio"]["enabled"] is (overlay is None)
    cfg = loki["loki"]
    assert cfg["schemaConfig"]["configs"][0]["object_store"] == "s3"
    assert cfg["compactor"]["retention_enabled"] and cfg["compactor"]["delete_request_store"] == "s3"
    assert cfg["limits_config"]["retention_period"] == "168h"
    labels = cfg["distributor"]["otlp_config"]["default_resource_attributes_as_index_labels"]
    assert {"k8s.namespace.name", "k8s.pod.name", "service.name"} <= set(labels)
    if overlay:
        aws = cfg["storage_config"]["aws"]
        assert {"region", "bucketnames", "access_key_id", "secret_access_key"} <= set(aws)
        # credentials are expanded from the Secret at start-up, never rendered into the config
        assert aws["access_key_id"] == "${AWS_ACCESS_KEY_ID}"
        assert aws["secret_access_key"] == "${AWS_SECRET_ACCESS_KEY}"
        for target in ("write", "read", "backend"):
            t = loki[target]
            assert "-config.expand-env=true" in t["extraArgs"]
            assert t["extraEnvFrom"][0]["secretRef"]["name"] == "loki-s3-credentials"
    otel = v["otelcol-logs"]
    assert otel["mode"] == "daemonset" and otel["podMonitor"]["enabled"]
    assert otel["podMonitor"]["extraLabels"]["release"] == "observability"
    hdr = otel["config"]["extensions"]["headers_setter/tenant"]["headers"][0]
    assert hdr["key"] == "X-Scope-OrgID" and hdr["value"] == v["tenant"]
    exp = otel["config"]["exporters"]["otlphttp/loki"]
    assert exp["endpoint"].startswith("http://loki-write.") and exp["endpoint"].endswith("/otlp")
    assert exp["auth"]["authenticator"] == "headers_setter/tenant"
    docs = helm_lite.render_chart(base, [os.path.join(base, overlay)] if overlay else [], {},
                                  release="logs-stack", namespace="observability")
    ds = [d for d in docs if d["kind"] == "ConfigMap"][0]
    body = yaml.safe_load(ds["data"]["loki.yaml"])["datasources"][0]
    assert body["url"] == "http://loki-read.observability:3100"
    assert body["jsonData"]["httpHeaderName1"] == "X-Scope-OrgID"
    assert body["secureJsonData"]["httpHeaderValue1"] == v["tenant"]


def test_observability_plays_apply_s3_overlay():
    """Both observability plays layer aws-s3-values.yaml (+ bucket / region / credentials)
    exactly when aws_access_key is set, and MinIO otherwise."""
    import yaml
    for play in ("deploy-observability.yml", "deploy-observability-openshift.yml"):
        doc = yaml.safe_load(open(os.path.join(ROOT, "core", "playbooks", play)))[0]
        vs = doc["vars"]
        assert "aws_access_key" in vs["logs_s3"]
        assert "aws-s3-values.yaml" in vs["logs_values_files"] and "if logs_s3" in \
            vs["logs_values_files"]
        aws = vs["logs_s3_values"]["loki"]["loki"]["storage_config"]["aws"]
        assert "aws_bucket" in aws["bucketnames"]
        # the keys go to a Secret (no_log), never into helm values / the Loki ConfigMap
        assert "secret_access_key" not in aws and "access_key_id" not in aws
        assert "aws_secret_key" not in str(vs)
        sec = [t for t in doc["tasks"] if t.get("name", "").startswith("Loki S3 credentials")][0]
        assert sec["no_log"] is True and "logs_s3" in sec["when"]
        body = sec["kubernetes.core.k8s"]["definition"]
        assert body["metadata"]["name"] == "loki-s3-credentials"
        assert "aws_secret_key" in body["stringData"]["AWS_SECRET_ACCESS_KEY"]
        task = [t for t in doc["tasks"] if t.get("name") == "Logs stack (Loki + OTEL collector)"][0]
        assert task["no_log"] is True
        h = task["kubernetes.core.helm"]
        assert h["values_files"] == "{{ logs_values_files }}"
        assert "logs_s3_values" in str(h["values"]) and "logs_common_values" in str(h["values"])
        # tenant and write endpoint from one variable each (collector header == datasource)
        cv = vs["logs_common_values"]
        assert cv["tenant"] == "{{ logs_tenant }}"
        hdr = cv["otelcol-logs"]["config"]["extensions"]["headers_setter/tenant"]["headers"][0]
        assert hdr["value"] == "{{ logs_tenant }}"
        ep = cv["otelcol-logs"]["config"]["exporters"]["otlphttp/loki"]["endpoint"]
        assert "{{ obs_ns }}" in ep
