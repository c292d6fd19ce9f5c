# full GPU parity suite + bench + scan phase stamps (one gpurun call)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?; tail -3 gpurun_out/gputests.log; test $rc -eq 0 && timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1
