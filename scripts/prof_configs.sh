set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/configs_r5b
mkdir -p $out
timeout -k 10 240 bash scripts/rocprof.sh "$out/prof_c5" 8 -- python3 bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 5 --warmup 3 --no_infer --no_walk > "$out/prof_c5.log" 2>&1 &&
timeout -k 10 240 bash scripts/rocprof.sh "$out/prof_c5f8" 8 -- python3 bench.py --num_hidden 1280 --num_rnn_layers 7 --fp8 --steps 5 --warmup 3 --no_infer --no_walk > "$out/prof_c5f8.log" 2>&1 &&
timeout -k 10 240 bash scripts/rocprof.sh "$out/prof_1760" 8 -- python3 bench.py --cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 --steps 5 --warmup 3 --no_infer --no_walk > "$out/prof_1760.log" 2>&1
