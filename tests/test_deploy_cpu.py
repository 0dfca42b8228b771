"""Deployment layer checks (SURVEY §4 deploy tests): YAML validity of charts/playbooks/inventory,
model catalog consistency with the MI355X Helm values, and the bash libs (model selection,
config parsing, tag building) exercised through bash."""

from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

import pytest
import yaml

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "core")
CATALOG = os.path.join(ROOT, "inventory/metadata/vars/model_catalog.yml")

pytestmark = pytest.mark.skipif(shutil.which("bash") is None, reason="bash missing")


def _bash(script: str, **env) -> subprocess.CompletedProcess:
    e = dict(os.environ, CORE_DIR=ROOT, model_catalog_file=CATALOG, **env)
    pre = (f'source "{ROOT}/lib/models/model-catalog.sh"; '
           f'source "{ROOT}/lib/models/model-selection.sh"; '
           f'source "{ROOT}/lib/models/install-model.sh"; '
           f'source "{ROOT}/lib/system/precheck/read-config-file.sh"; ')
    return subprocess.run(["bash", "-c", pre + script], capture_output=True, text=True, env=e,
                          timeout=60)


def test_all_yaml_parses():
    files = [f for f in glob.glob(ROOT + "/**/*.y*ml", recursive=True) if "/templates/" not in f]
    assert len(files) > 30
    for f in files:
        list(yaml.safe_load_all(open(f)))


def test_all_shell_scripts_syntax():
    for f in glob.glob(ROOT + "/**/*.sh", recursive=True):
        r = subprocess.run(["bash", "-n", f], capture_output=True, text=True)
        assert r.returncode == 0, (f, r.stderr)


def test_catalog_consistent_with_values():
    cat = yaml.safe_load(open(CATALOG))["model_catalog"]
    nums = [m["number"] for m in cat]
    assert len(set(nums)) == len(nums)
    assert len({m["release"] for m in cat}) == len(cat)
    vals = yaml.safe_load(open(os.path.join(ROOT, "helm-charts/vllm/mi355x-values.yaml")))
    cfgs = vals["modelConfigs"]
    for m in cat:
        assert m["chart"] in ("vllm", "tei", "teirerank")
        assert m["platform"] in ("gpu", "cpu")
        if m["chart"] == "vllm" and m["platform"] == "gpu":
            assert m["model_id"] in cfgs, m["model_id"]
            assert 1 <= m["tensor_parallel_size"] <= 8
    # the flagship serving config runs one MI355X per Llama-3.1-8B replica
    assert next(m for m in cat if m["name"] == "llama-8b")["tensor_parallel_size"] == 1


def test_catalog_models_resolve_in_framework():
    """Every GPU LLM in the catalog maps to a model class this framework implements."""
    from enterprise_inference_amd.models import catalog as mc
    cat = yaml.safe_load(open(CATALOG))["model_catalog"]
    for m in cat:
        if m["chart"] != "vllm":
            continue
        assert mc.get_preset(m["model_id"])["architectures"], m["model_id"]


def test_get_model_names_gpu_and_cpu():
    r = _bash("get_model_names", models="1,2", cpu_or_gpu="g")
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["llama-8b", "llama-70b"]
    r = _bash("get_model_names", models="1", cpu_or_gpu="c")
    assert r.returncode != 0 and "GPU model identifier" in r.stderr
    r = _bash("get_model_names", models="x", cpu_or_gpu="g")
    assert r.returncode != 0 and "invalid" in r.stderr
    r = _bash("get_model_names", models="999", cpu_or_gpu="g")
    assert r.returncode != 0 and "unknown" in r.stderr


def test_build_model_tags():
    r = _bash("build_model_tags install", model_name_list="llama-8b llama-70b",
              deploy_genai_gateway="yes", deploy_keycloak="no", huggingface_model_deployment_name="")
    assert r.stdout.strip() == "install-llama-8b,install-llama-70b,install-genai-gateway"
    r = _bash("build_model_tags uninstall", model_name_list="llama-8b",
              deploy_genai_gateway="yes", huggingface_model_deployment_name="my-model")
    assert r.stdout.strip() == "uninstall-llama-8b,uninstall-my-model"


def test_read_config_file_and_platform(tmp_path):
    cfg = tmp_path / "inference-config.cfg"
    cfg.write_text("cluster_url=api.example.com\ncpu_or_gpu=mi355x  # comment\n"
                   "deploy_keycloak_apisix=on\ndeploy_observability=off\n")
    r = _bash(f'read_config_file "{cfg}" && '
              'echo "$cluster_url|$cpu_or_gpu|$gpu_platform|$deploy_observability"')
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == "api.example.com|g|mi355x|no"
    cfg.write_text("cpu_or_gpu=gaudi3\n")
    r = _bash(f'read_config_file "{cfg}" && normalise_platform')
    assert r.returncode != 0
    cfg.write_text("cpu_or_gpu=mi300x\n")
    r = _bash(f'read_config_file "{cfg}" && normalise_platform && echo "$cpu_or_gpu $gpu_platform"')
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == "g mi300x"


def test_playbook_file_references_exist():
    """Files a playbook names under helm_charts_base / tasks/ exist in the tree."""
    import re
    pb_dir = os.path.join(ROOT, "playbooks")
    for f in glob.glob(pb_dir + "/*.yml") + glob.glob(pb_dir + "/tasks/*.yml"):
        s = open(f).read()
        for rel in re.findall(r"(?<!remote_)helm_charts_base(?: ~ '|\s*}}\s*)(/[\w./-]+)", s):
            assert os.path.exists(os.path.join(ROOT, "helm-charts") + rel.rstrip("'")), (f, rel)
        for inc in re.findall(r"include_tasks:\s*([\w./-]+\.yml)", s):
            base = os.path.dirname(f)
            assert os.path.exists(os.path.join(base, inc)), (f, inc)


def test_istio_and_ceph_flow_wiring():
    istio = open(os.path.join(ROOT, "lib/components/istio.sh")).read()
    assert "deploy-istio-openshift.yml" in istio and "deploy-istio.yml" in istio
    ceph = open(os.path.join(ROOT, "lib/components/ceph.sh")).read()
    assert ceph.index("generate-ceph-values.yml") < ceph.index("deploy-ceph-storage.yml")
    pa = list(yaml.safe_load_all(open(os.path.join(ROOT, "helm-charts/istio/peer-auth-ingress.yaml"))))
    assert pa[0]["spec"]["portLevelMtls"][443]["mode"] == "PERMISSIVE"


def test_ibm_pattern_files():
    d = os.path.join(os.path.dirname(ROOT), "third_party/IBM/patterns/quickstart")
    for f in ("main.tf", "variables.tf", "versions.tf", "inference-config.tpl", "run_script.sh",
              "templates/inventory.yaml.tftpl"):
        assert os.path.exists(os.path.join(d, f)), f
    r = subprocess.run(["bash", "-n", os.path.join(d, "run_script.sh")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # every ${var} of the config template is supplied by main.tf's templatefile() call
    import re
    tpl_vars = set(re.findall(r"\$\{(\w+)\}", open(os.path.join(d, "inference-config.tpl")).read()))
    main = open(os.path.join(d, "main.tf")).read()
    block = main[main.index('templatefile("${path.module}/inference-config.tpl"'):]
    block = block[:block.index("})")]
    assert tpl_vars <= set(re.findall(r"^\s*(\w+)\s*=", block, re.M)), tpl_vars
    # keys written into inference-config.cfg are ones the installer reads
    cfg_keys = {l.split("=")[0] for l in open(os.path.join(ROOT, "inventory/inference-config.cfg"))
                if "=" in l}
    tpl_keys = {l.split("=")[0] for l in open(os.path.join(d, "inference-config.tpl")) if "=" in l}
    assert tpl_keys <= cfg_keys, tpl_keys - cfg_keys


def test_ibm_standard_pattern_and_catalog():
    """The standard flavor creates its own network and reuses the quickstart templates; the
    catalog manifest lists every Terraform input of both flavors (generated, never stale)."""
    import re
    base = os.path.join(os.path.dirname(ROOT), "third_party/IBM/patterns")
    main = open(os.path.join(base, "standard/main.tf")).read()
    for res in ("ibm_is_vpc", "ibm_is_security_group", "ibm_is_public_gateway", "ibm_is_subnet"):
        assert f'resource "{res}"' in main, res
    assert "data \"ibm_is_vpc\"" not in main
    for ref in re.findall(r'\$\{path\.module\}/([\w./-]+)', main):
        assert os.path.exists(os.path.join(base, "standard", ref)), ref
    # every var.X used by the pattern is declared
    decl = set(re.findall(r'variable "(\w+)"', open(os.path.join(base, "standard/variables.tf")).read()))
    used = set(re.findall(r"\bvar\.(\w+)", main))
    assert used <= decl, used - decl
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(ROOT), "scripts/gen_ibm_catalog.py"),
                        "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_multi_node_example():
    d = os.path.join(os.path.dirname(ROOT), "docs/examples/multi-node")
    inv = yaml.safe_load(open(os.path.join(d, "hosts.yaml")))
    ch = inv["all"]["children"]
    cps = set(ch["kube_control_plane"]["hosts"])
    assert len(cps) == 3 and set(ch["etcd"]["hosts"]) == cps
    workers = set(ch["kube_node"]["hosts"])
    assert workers and not (workers & cps)
    assert all(inv["all"]["hosts"][w].get("devices") for w in workers)
    cfg_keys = {l.split("=")[0] for l in open(os.path.join(ROOT, "inventory/inference-config.cfg"))
                if "=" in l}
    ex_keys = {l.split("=")[0] for l in open(os.path.join(d, "inference-config.cfg")) if "=" in l}
    assert ex_keys == cfg_keys


# --------------------------------------------------------------------------- variable wiring

def _checker():
    sys.path.insert(0, os.path.join(os.path.dirname(ROOT), "scripts"))
    import check_playbook_vars
    return check_playbook_vars


def test_every_playbook_renders_with_strict_undefined():
    """Every play's Jinja (tasks, included task files, roles, role templates, the Langfuse
    values template) renders against group vars + vars files + the GENERATED vault + the
    --extra-vars the CLI passes that playbook, with StrictUndefined."""
    ch = _checker().Checker(ROOT)
    for pb in sorted(glob.glob(os.path.join(ROOT, "playbooks/*.yml"))):
        ch.check_playbook(pb)
    assert ch.errors == [], "\n".join(ch.errors)


def test_strict_render_catches_a_missing_vault(tmp_path):
    """The round-1 bug: the gateway play used vault secrets without loading the vault."""
    core = tmp_path / "core"
    shutil.copytree(ROOT, core)
    pb = core / "playbooks/deploy-genai-gateway.yml"
    pb.write_text(pb.read_text().replace("    - ../config/vault.yml\n", ""))
    ch = _checker().Checker(str(core))
    ch.check_playbook(str(pb))
    assert any("litellm_master_key" in e for e in ch.errors), ch.errors


def _keys(d, prefix=""):
    out = set()
    for k, v in d.items():
        out.add(prefix + k)
        if isinstance(v, dict):
            out |= _keys(v, prefix + k + ".")
    return out


def test_gateway_play_values_exist_in_chart():
    """Every value the play passes to the genai-gateway chart is a key the chart defines
    (round 1 passed masterKey / postgres.password to a chart reading masterkey / postgresql)."""
    chart = yaml.safe_load(open(os.path.join(ROOT, "helm-charts/genai-gateway/values.yaml")))
    play = yaml.safe_load(open(os.path.join(ROOT, "playbooks/deploy-genai-gateway.yml")))[0]
    task = next(t for t in play["tasks"] if t.get("name") == "Gateway chart")
    passed = _keys(task["kubernetes.core.helm"]["values"])
    missing = sorted(k for k in passed if k not in _keys(chart))
    assert missing == [], missing
    tmpl = open(os.path.join(ROOT, "helm-charts/genai-gateway/templates/deployment.yaml")).read()
    assert "wait-for-postgres-restore" in tmpl and "kubectl" in tmpl
    restore = open(os.path.join(ROOT, "helm-charts/genai-gateway/templates/postgres-restore-job.yaml")).read()
    assert "n_live_tup" in restore       # restores only into an empty database


def test_vault_generator_has_reference_keys(tmp_path):
    out = tmp_path / "vault.yml"
    subprocess.run(["bash", os.path.join(ROOT, "scripts/generate-vault-secrets.sh"), str(out)],
                   check=True, capture_output=True)
    v = yaml.safe_load(out.read_text())
    ref = ["litellm_master_key", "litellm_salt_key", "redis_password", "langfuse_secret_key",
           "langfuse_public_key", "postgresql_username", "postgresql_password",
           "clickhouse_username", "clickhouse_password", "langfuse_login", "langfuse_user",
           "langfuse_password", "minio_secret", "minio_user", "postgres_user", "postgres_password",
           "grafana_admin_password"]
    assert all(v.get(k) for k in ref), [k for k in ref if not v.get(k)]
    assert oct(out.stat().st_mode & 0o777) == "0o600"


def _topology_mod():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "topology", os.path.join(ROOT, "roles/utils/get_optimized_cpu_topology/files/topology.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _topo(sockets, numa_per_socket, cpus_per_numa, free_gb_per_numa, amx=False):
    numa, c = [], 0
    for s in range(sockets):
        for j in range(numa_per_socket):
            numa.append({"node": s * numa_per_socket + j, "socket": s,
                         "cpus": list(range(c, c + cpus_per_numa)),
                         "mem_total_kb": int(free_gb_per_numa * 1.2 * 1048576),
                         "mem_free_kb": int(free_gb_per_numa * 1048576), "gpus": []})
            c += cpus_per_numa
    return {"numa": numa, "sockets": sockets, "amx": amx, "avx512": True, "avx2": True}


@pytest.mark.parametrize("sockets,nps,want_tp,want_pp", [(2, 2, 2, 2), (2, 3, 2, 2), (1, 4, 4, 1),
                                                          (2, 6, 4, 2), (1, 1, 1, 1), (2, 1, 1, 2)])
def test_cpu_topology_plan_rules(sockets, nps, want_tp, want_pp):
    """Reference rules (get_optimized_cpu_topology.yaml:407-420, :503-521): TP from NUMA nodes
    per socket, 18 % of a socket's CPUs reserved (>= 2, <= half), 82 % of free memory."""
    t = _topology_mod()
    p = t.plan(_topo(sockets, nps, 24, 100.0, amx=True))
    cps = 24 * nps
    assert p["tensor_parallel_size"] == want_tp and p["pipeline_parallel_size"] == want_pp
    reserved = max(2, min(-(-cps * 18 // 100), cps // 2))
    assert p["reserved_cpus_per_socket"] == reserved
    expect_balloon = (cps - reserved) // 2 if (sockets == 1 and nps == 1) else cps - reserved
    assert p["balloon_cpus"] == expect_balloon
    assert p["memory_gi"] == int(100.0 * nps * 0.82)
    assert p["isa"] == "amx"
    assert len(p["reserved_cpuset"].split(",")) == reserved * sockets


def test_topology_probe_reads_sysfs(tmp_path):
    """probe() on a synthetic /sys + /proc tree (2 NUMA nodes, one MI355X on node 1)."""
    t = _topology_mod()
    for n, cpus in ((0, "0-3"), (1, "4-7")):
        d = tmp_path / f"sys/devices/system/node/node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus)
        (d / "meminfo").write_text(f"Node {n} MemTotal: 1048576 kB\nNode {n} MemFree: 524288 kB\n")
    for c in range(8):
        d = tmp_path / f"sys/devices/system/cpu/cpu{c}/topology"
        d.mkdir(parents=True)
        (d / "physical_package_id").write_text("0")
        (d / "thread_siblings_list").write_text(str(c))
    g = tmp_path / "sys/bus/pci/devices/0000:05:00.0"
    g.mkdir(parents=True)
    (g / "vendor").write_text("0x1002")
    (g / "class").write_text("0x120000")
    (g / "numa_node").write_text("1")
    (tmp_path / "proc").mkdir()
    (tmp_path / "proc/cpuinfo").write_text("flags : fpu avx2 avx512f\n")
    topo = t.probe(str(tmp_path))
    assert [len(n["cpus"]) for n in topo["numa"]] == [4, 4]
    assert topo["numa"][1]["gpus"] == ["0000:05:00.0"] and topo["avx512"]
    p = t.plan(topo)
    assert p["tensor_parallel_size"] == 2 and p["gpu_numa"] == {"1": ["0000:05:00.0"]}


def test_nri_balloon_matches_vllm_pods():
    import jinja2
    tmpl = open(os.path.join(ROOT, "roles/nri_cpu_balloons/templates/balloons-values.yaml.j2")).read()
    d = yaml.safe_load(open(os.path.join(ROOT, "roles/nri_cpu_balloons/defaults/main.yml")))
    out = jinja2.Environment(undefined=jinja2.StrictUndefined).from_string(tmpl).render(
        cpu_parallelism={"balloon_cpus": 40, "reserved_cpuset": "0,1,2,3"}, **d)
    cfg = yaml.safe_load(out)["config"]
    bt = cfg["balloonTypes"][0]
    assert bt["name"] == "vllm-balloon" and bt["minCPUs"] == 40
    assert bt["matchExpressions"] == [{"key": "name", "operator": "In", "values": ["vllm"]}]
    assert cfg["reservedResources"]["cpu"] == "cpuset:0,1,2,3"
    dep = open(os.path.join(ROOT, "helm-charts/vllm/templates/deployment.yaml")).read()
    assert "name: vllm" in dep           # the pod label the balloon matches
