#!/usr/bin/env bash
# Update the amdgpu DKMS kernel driver and/or GPU firmware on one node (run by
# playbooks/deploy-amdgpu-driver-firmware.yml).  Compares the installed versions
# reported by amd-smi / dkms with the target and only acts when they differ.
# Usage: amdgpu-driver-firmware-updater.sh --drivers|--firmware|--both <rocm_version> <driver_version>
set -euo pipefail
mode=${1:---both}; rocm=${2:-7.2.0}; drv=${3:-}
log() { echo "[amdgpu-updater] $*"; }
installed_driver() { dkms status amdgpu 2>/dev/null | awk -F'[ ,/:]+' '/amdgpu/{print $2; exit}'; }
update_driver() {
  local cur; cur=$(installed_driver || true)
  if [ -n "$drv" ] && [ "$cur" = "$drv" ]; then log "driver $cur already installed"; return 0; fi
  log "installing amdgpu-dkms (ROCm ${rocm}) over '${cur:-none}'"
  . /etc/os-release
  # pinned to the metadata driver version when one is given (apt / dnf version globs)
  case "$ID" in
    ubuntu) apt-get update -y && apt-get install -y --allow-downgrades "amdgpu-dkms${drv:+=1:${drv}*}" ;;
    rhel|rocky|almalinux) dnf install -y "amdgpu-dkms${drv:+-${drv}*}" ;;
    *) log "unsupported OS $ID"; return 1 ;;
  esac
  log "reloading the amdgpu module (GPU workloads on this node must be drained)"
  if ! (modprobe -r amdgpu && modprobe amdgpu); then
    log "module in use: reboot required"
  fi
}
update_firmware() {
  log "current firmware:"; amd-smi firmware 2>/dev/null | head -40 || true
  if command -v amd-smi >/dev/null 2>&1 && amd-smi firmware --help 2>/dev/null | grep -q update; then
    amd-smi firmware update --all
  else
    log "installing amdgpu firmware package"
    . /etc/os-release
    case "$ID" in
      ubuntu) apt-get install -y --only-upgrade linux-firmware amdgpu-dkms-firmware || true ;;
      *) dnf upgrade -y linux-firmware || true ;;
    esac
  fi
}
case "$mode" in
  --drivers) update_driver ;;
  --firmware) update_firmware ;;
  --both) update_driver && update_firmware ;;
  *) echo "usage: $0 --drivers|--firmware|--both [rocm_version] [driver_version]"; exit 2 ;;
esac
log "done"
