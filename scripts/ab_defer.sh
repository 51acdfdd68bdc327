set -o pipefail
mkdir -p gpurun_out/ab
r() { timeout -k 10 120 env "$@" > gpurun_out/ab/$(echo "$*" | tr ' =/-' '____').log 2>&1; }
for i in 1 2; do
r DS2_DEFER_DW=1 python bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 15 --warmup 5 &&
r DS2_DEFER_DW=0 python bench.py --num_hidden 1280 --num_rnn_layers 7 --steps 15 --warmup 5 &&
r DS2_DEFER_DW=1 python bench.py --cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 --steps 15 --warmup 5 &&
r DS2_DEFER_DW=0 python bench.py --cell rnn_relu --num_hidden 1760 --num_rnn_layers 7 --steps 15 --warmup 5 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/*.log
