set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 ./tools/_stencil_probe > gpurun_out/stencil_probe.log 2>&1; st=$?; cat gpurun_out/stencil_probe.log; exit $st
