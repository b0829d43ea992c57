# Round-6 close-out check on one MI355X: build() output as shipped, smoke(), the whole GPU suite
set -o pipefail
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r6.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r6.txt
exit $rc
