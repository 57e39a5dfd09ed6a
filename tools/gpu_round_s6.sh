#!/bin/bash
# r02_s6 round pass: tests, smoke, 70k / 256k / C5 benches, rocprof kernel stats, then PMC traffic passes
bash tools/gpu_round.sh r02_s6 || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_bench.sh r02_s6_pmc || exit $?
python tools/pmc_summary.py gpurun_out/r02_s6_pmc > gpurun_out/r02_s6_pmc/summary.txt
python -c "import sys; sys.path.insert(0, 'tools'); import pmc_summary as p; p.traffic_json('gpurun_out/r02_s6_pmc', 'gpurun_out/r02_s6_pmc/pmc_traffic.json', 70000, 'r02_s6')"
