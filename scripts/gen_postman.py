#!/usr/bin/env python3
"""Generate the Postman collection (core/catalog/) from the model catalog: a Keycloak token
request plus, per deployable model, requests for both gateway modes -- APISIX routes
(``https://{{cluster_url}}/<last id segment>/v1/...`` with the Keycloak bearer token) and the
LiteLLM GenAI gateway (``/v1/...`` with the gateway key).  Mirrors the reference's manual API
smoke tests (core/catalog/AI-Inference-as-Service-postman-collection.json)."""
import json
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CATALOG = os.path.join(ROOT, "core/inventory/metadata/vars/model_catalog.yml")
OUT = os.path.join(ROOT, "core/catalog/AI-Inference-MI355X.postman_collection.json")


def req(name, url_path, body, auth_var, method="POST"):
    return {"name": name, "request": {
        "method": method,
        "header": [{"key": "Content-Type", "value": "application/json"},
                   {"key": "Authorization", "value": "Bearer {{%s}}" % auth_var}],
        "body": {"mode": "raw", "raw": json.dumps(body, indent=2)},
        "url": {"raw": "https://{{cluster_url}}" + url_path, "protocol": "https",
                "host": ["{{cluster_url}}"], "path": [p for p in url_path.split("/") if p]}}}


def model_requests(m, auth_var, prefix):
    mid = m["model_id"]
    if m["mode"] == "embedding":
        return [req(f"{m['name']} embeddings", f"{prefix}/v1/embeddings",
                    {"model": mid, "input": ["What is deep learning?"]}, auth_var)]
    if m["mode"] == "rerank":
        path = f"{prefix}/rerank" if prefix else "/v1/rerank"
        return [req(f"{m['name']} rerank", path,
                    {"model": mid, "query": "What is deep learning?",
                     "texts": ["Deep learning is a subset of ML.", "Paris is in France."]},
                    auth_var)]
    return [
        req(f"{m['name']} chat", f"{prefix}/v1/chat/completions",
            {"model": mid, "messages": [{"role": "user", "content": "What is deep learning?"}],
             "max_tokens": 64, "temperature": 0}, auth_var),
        req(f"{m['name']} completions (stream)", f"{prefix}/v1/completions",
            {"model": mid, "prompt": "What is deep learning?", "max_tokens": 64, "stream": True,
             "stream_options": {"include_usage": True}}, auth_var),
    ]


def main():
    cat = yaml.safe_load(open(CATALOG))["model_catalog"]
    token = {"name": "Get Keycloak token", "event": [{"listen": "test", "script": {"exec": [
        "pm.environment.set('access_token', pm.response.json().access_token);"]}}],
        "request": {"method": "POST", "header": [{"key": "Content-Type",
                                                  "value": "application/x-www-form-urlencoded"}],
                    "body": {"mode": "urlencoded", "urlencoded": [
                        {"key": "grant_type", "value": "client_credentials"},
                        {"key": "client_id", "value": "{{keycloak_client_id}}"},
                        {"key": "client_secret", "value": "{{keycloak_client_secret}}"}]},
                    "url": {"raw": "https://{{cluster_url}}/token", "protocol": "https",
                            "host": ["{{cluster_url}}"], "path": ["token"]}}}
    apisix, gw = [token], []
    for m in cat:
        seg = m["model_id"].split("/")[-1]
        if m["platform"] == "cpu":
            seg += "-vllmcpu"
        apisix += model_requests(m, "access_token", f"/{seg}")
        gw += model_requests(m, "litellm_api_key", "")
    coll = {"info": {"name": "AI Inference as a Service -- AMD Instinct MI355X",
                     "schema": "https://schema.getpostman.com/json/collection/v2.1.0/collection.json"},
            "variable": [{"key": "cluster_url", "value": "api.example.com"},
                         {"key": "keycloak_client_id", "value": "my-client-id"},
                         {"key": "keycloak_client_secret", "value": ""},
                         {"key": "litellm_api_key", "value": ""}],
            "item": [{"name": "Keycloak + APISIX", "item": apisix},
                     {"name": "GenAI gateway (LiteLLM)", "item": gw}]}
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(coll, f, indent=2)
    print(OUT, sum(len(g["item"]) for g in coll["item"]), "requests")


if __name__ == "__main__":
    main()
