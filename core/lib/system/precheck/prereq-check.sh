#!/usr/bin/env bash
# Host prerequisites for the deploy node: git, python>=3.10, curl, pip, venv.
run_system_prerequisites_check() {
    local missing=()
    for tool in git curl python3; do
        command -v "$tool" >/dev/null 2>&1 || missing+=("$tool")
    done
    if command -v python3 >/dev/null 2>&1; then
        if ! python3 -c 'import sys; sys.exit(0 if sys.version_info >= (3, 10) else 1)'; then
            echo "python3 >= 3.10 is required" >&2
            return 1
        fi
        python3 -m venv --help >/dev/null 2>&1 || missing+=("python3-venv")
        python3 -m pip --version >/dev/null 2>&1 || missing+=("python3-pip")
    fi
    if [ ${#missing[@]} -gt 0 ]; then
        echo "Missing prerequisites: ${missing[*]}"
        if command -v apt-get >/dev/null 2>&1; then
            while fuser /var/lib/dpkg/lock-frontend >/dev/null 2>&1; do sleep 5; done
            sudo apt-get update -y && sudo apt-get install -y "${missing[@]}" || return 1
        elif command -v dnf >/dev/null 2>&1; then
            sudo dnf install -y "${missing[@]}" || return 1
        else
            return 1
        fi
    fi
    return 0
}
