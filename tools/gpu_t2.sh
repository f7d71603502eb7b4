timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_t2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_t2.log; [ $rc -eq 0 ] || exit 3
VXG_PLAN_DEBUG=1 timeout -k 10 300 python -u bench.py --workloads c3,c5 --no-cpu-baseline > gpurun_out/bench_c35_t2.json 2> gpurun_out/bench_c35_t2.err || exit 4
VXG_PLAN_DEBUG=1 timeout -k 10 300 python -u bench.py --workloads c3,c5 --no-cpu-baseline --simulate-world 8 > gpurun_out/bench_sim8_t2.json 2> gpurun_out/bench_sim8_t2.err || exit 4
bash tools/gpu_c5traffic.sh t2
