#!/usr/bin/env bash
# Client-credentials access token through the gateway's /token route.
# Usage: generate-token.sh <cluster_url> <client_id> <client_secret>
set -euo pipefail
curl -sk -X POST "https://$1/token" -d grant_type=client_credentials -d "client_id=$2" \
  -d "client_secret=$3" | python3 -c 'import json,sys; print(json.load(sys.stdin)["access_token"])'
