

def test_batch_validate_rejects_overlong_labels():
    """Host-side length checks before upload (the CTC kernels only clamp)."""
    import numpy as np
    import pytest
    from deepspeech_amd.data.synthetic import Batch
    ok = Batch(np.zeros((2, 10, 4), np.float32), np.array([10, 7], np.int32),
               np.zeros((2, 3), np.int32), np.array([3, 1], np.int32))
    assert ok.validate() is ok
    with pytest.raises(ValueError, match="label length"):
        Batch(ok.feats, ok.seq_lens, ok.labels, np.array([4, 1], np.int32)).validate()
    with pytest.raises(ValueError, match="sequence length"):
        Batch(ok.feats, np.array([11, 1], np.int32), ok.labels, ok.label_lens).validate()
