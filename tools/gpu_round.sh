# one GPU call: profile the default kernel, then the bench line
set -u
bash tools/profile.sh $1 --frames 5 > gpurun_out/prof_$1.log 2>&1; echo prof_rc=$?
timeout -k 10 600 python bench.py > gpurun_out/bench_$1.json 2> gpurun_out/bench_$1.err; echo bench_rc=$?
cat gpurun_out/bench_$1.json
