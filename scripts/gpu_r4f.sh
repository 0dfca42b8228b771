#!/bin/bash
# Round-4 kernels in one box session: stream-K decode (r4d) + prefill FA / wide add+norm (r4e).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash scripts/gpu_r4e.sh && bash scripts/gpu_r4d.sh
