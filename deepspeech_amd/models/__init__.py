from .deepspeech2 import DeepSpeech2, build_model, conv_out_len, freq_out, GATES  # noqa: F401
