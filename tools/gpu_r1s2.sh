set -o pipefail
mkdir -p gpurun_out/r1s2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1s2/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1s2/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r1s2/bench.json 2> gpurun_out/r1s2/bench.err
