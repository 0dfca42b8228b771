#!/usr/bin/env bash
# Run one workflow step; print a coloured verdict and stop the whole run on failure.
execute_and_check() {
    local description=$1
    shift
    echo "${BLUE:-}==> ${description}${NC:-}"
    if "$@"; then
        echo "${GREEN:-}[ok] ${description}${NC:-}"
    else
        local rc=$?
        echo "${RED:-}[failed rc=${rc}] ${description}${NC:-}" >&2
        exit 1
    fi
}
