#!/bin/bash
# Diagnostic: the GPU suite with every kernel launch and copy serialised and error-checked by the
# HIP runtime (AMD_SERIALIZE_KERNEL / AMD_SERIALIZE_COPY = 3), so a device fault is reported at the
# launch or copy that caused it instead of at a later API call. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/diag
export AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread \
  > gpurun_out/diag/pytest_gpu_serialized.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/diag/pytest_gpu_serialized.log
exit $rc
