timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k4.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k4.log; [ $rc -eq 0 ] || exit 3
bash tools/gpu_c5plan.sh k4 && bash tools/gpu_shard_prof.sh k4
