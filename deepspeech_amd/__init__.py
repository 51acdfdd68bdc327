"""deepspeech_amd — a DeepSpeech2 training / inference engine built for AMD Instinct MI355X.

Capability parity target: yxlao/deepSpeech (TensorFlow 1.x DeepSpeech2 for Intel CPUs).
The compute path is PyTorch-ROCm plus hand-written CDNA4 (gfx950) HIP kernels in
``deepspeech_amd/csrc``; data-parallel scaling uses ``torch.distributed`` over RCCL.

Layer map (see SURVEY.md §1 for the reference's):
  models/    DeepSpeech2 network (conv front-end, recurrent stack, FC head)
  ops/       autograd wrappers around the HIP kernels + pure-torch reference ops
  parallel/  process-group setup, bucketed gradient all-reduce overlapped with backward
  data/      synthetic / TFRecord / bucketed SortaGrad input pipelines, featurizer
  utils/     checkpoints, metrics, LR schedule, profiling, summaries
  runtime/   native (C++) host runtime: loader threads, beam search, TFRecord codec
"""

__version__ = "0.1.0"

# Character set and class count (reference: src/deepSpeech_input.py:13-14).
ALPHABET = "ABCDEFGHIJKLMNOPQRSTUVWXYZ' "
NUM_CLASSES = len(ALPHABET) + 1  # + CTC blank
BLANK = NUM_CLASSES - 1          # TF's ctc_loss uses the last class as blank
FREQ_BINS = 161                  # spectrogram / "mfcc" bins (src/deepSpeech_input.py:42)
