set -u
mkdir -p gpurun_out/b2
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/b2/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/b2/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/b2/rocprof.log 2>&1
