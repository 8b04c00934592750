source tools/gpu_steps.sh
mkdir -p /tmp/bp && hipcc --offload-arch=gfx950 -O2 tools/probe/sync_cpu_probe.hip -o /tmp/bp/sync_cpu_probe 2>/dev/null
step sync_default 60 /tmp/bp/sync_cpu_probe blocking
ROC_ACTIVE_WAIT_TIMEOUT=0 step sync_awt0 60 /tmp/bp/sync_cpu_probe blocking
ROC_ACTIVE_WAIT_TIMEOUT=5 step sync_awt5 60 /tmp/bp/sync_cpu_probe blocking
ROC_ACTIVE_WAIT_TIMEOUT=20 step sync_awt20 60 /tmp/bp/sync_cpu_probe blocking
