# Shared by train.sh / test.sh / validation.sh (reference: src/train.sh:21-38).
# Config-combination guard: the reference accepts (NHWC x {tf, cudnn_rnn}) or
# (NCHW x {mkl, mkldnn_rnn}); here every engine runs in either layout, so the guard only
# rejects unknown values: engine in {hip, ref, tf, mkl, cudnn_rnn, mkldnn_rnn} (the
# reference names alias onto hip / ref), nchw/dummy/debug in {True, False}.
check_config() {
  case "${engine}" in hip|ref|tf|mkl|cudnn_rnn|mkldnn_rnn) ;; *) echo "unsupported engine ${engine}"; exit 1;; esac
  for v in "${nchw}" "${dummy:-False}" "${debug:-False}"; do
    case "$v" in True|False) ;; *) echo "unsupported configuration combination ($v)"; exit 1;; esac
  done
}
repo_root=$(cd "$(dirname "$0")/.." && pwd)
export PYTHONPATH=${repo_root}:${PYTHONPATH}
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
