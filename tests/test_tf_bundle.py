"""TF Saver-V2 checkpoint bundles (utils/tf_bundle.py + runtime/tensor_bundle.cpp).

The reference saves and restores ``model.ckpt-<step>.{index,data-00000-of-00001}`` with
tf.train.Saver (src/deepSpeech_train.py:354-356, :383-398, :471; eval restores the EMA shadows,
src/deepSpeech_test.py:93-109, :217-220). TensorFlow is not importable here and the reference
ships no checkpoint, so parity with TF-written files is UNPINNED; these tests pin the format
against an independent pure-Python implementation of the published layout (LevelDB table
format + the BundleHeaderProto / BundleEntryProto wire encoding) in both directions, plus round
trips, checksums and corruption detection."""
import os
import struct

import pytest
import torch

from deepspeech_amd.runtime import native
from deepspeech_amd.utils import tf_bundle as TB

pytestmark = pytest.mark.skipif(not native.available(), reason="native runtime not built")


# ---- an independent implementation of the on-disk format (spec, not our code) -------------
def _crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def _mask(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(v: int) -> bytes:
    out = b""
    while v >= 0x80:
        out += bytes([(v & 0x7F) | 0x80])
        v >>= 7
    return out + bytes([v])


def _read_varint(b: bytes, i: int):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7F) << s
        if x < 0x80:
            return r, i
        s += 7


def _spec_block(entries, restart_every):
    """LevelDB block: shared/unshared/value-length varints, restarts, restart count."""
    out, restarts, last = b"", [], b""
    for j, (k, v) in enumerate(entries):
        if j % restart_every == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        last = k
    for r in restarts or [0]:
        out += struct.pack("<I", r)
    return out + struct.pack("<I", len(restarts or [0]))


def _spec_table(entries, per_block=3):
    """A table with several small data blocks (the writer under test uses 256 KiB blocks)."""
    f = b""
    index = []

    def emit(block):
        nonlocal f
        off = len(f)
        f += block + b"\x00" + struct.pack("<I", _mask(_crc32c(block + b"\x00")))
        return off, len(block)
    for s in range(0, len(entries), per_block):
        chunk = entries[s:s + per_block]
        off, n = emit(_spec_block(chunk, 2))
        index.append((chunk[-1][0], _varint(off) + _varint(n)))
    moff, mn = emit(_spec_block([], 1))
    ioff, inn = emit(_spec_block(index, 1))
    footer = (_varint(moff) + _varint(mn) + _varint(ioff) + _varint(inn)).ljust(40, b"\x00")
    return f + footer + struct.pack("<Q", 0xDB4775248B80FB57)


def _spec_parse_table(f: bytes):
    assert struct.unpack("<Q", f[-8:])[0] == 0xDB4775248B80FB57
    ft = f[-48:-8]
    _, i = _read_varint(ft, 0)
    _, i = _read_varint(ft, i)
    ioff, i = _read_varint(ft, i)
    isz, i = _read_varint(ft, i)

    def block(off, n):
        b = f[off:off + n]
        assert f[off + n] == 0
        assert struct.unpack("<I", f[off + n + 1:off + n + 5])[0] == _mask(_crc32c(b + b"\x00"))
        nres = struct.unpack("<I", b[-4:])[0]
        end = len(b) - 4 - 4 * nres
        i, key, out = 0, b"", []
        while i < end:
            sh, i = _read_varint(b, i)
            un, i = _read_varint(b, i)
            vl, i = _read_varint(b, i)
            key = key[:sh] + b[i:i + un]
            i += un
            out.append((key, b[i:i + vl]))
            i += vl
        return out
    out = []
    for _, h in block(ioff, isz):
        off, j = _read_varint(h, 0)
        n, _ = _read_varint(h, j)
        out += block(off, n)
    return out


def _spec_entry(dtype_enum, shape, offset, size, crc):
    dims = b"".join(b"\x12" + _varint(len(d)) + d for d in (b"\x08" + _varint(x) for x in shape))
    return (b"\x08" + _varint(dtype_enum) + b"\x12" + _varint(len(dims)) + dims + b"\x20" + _varint(offset) +
            b"\x28" + _varint(size) + b"\x35" + struct.pack("<I", crc))


# ---- tests -------------------------------------------------------------------------------------
def test_crc32c_known_vectors():
    N = native.load()
    assert N.bundle_masked_crc32c(b"123456789") == _mask(0xE3069283)      # RFC 3720 check value
    buf = os.urandom(4099)
    assert N.bundle_masked_crc32c(buf) == _mask(_crc32c(buf))            # unaligned head / tail


def test_hand_built_bundle_parses(tmp_path):
    """An index + data shard assembled by hand from the format description (several data
    blocks, prefix-compressed keys, restart points) reads back through read_bundle."""
    a = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    g = torch.tensor(7, dtype=torch.int64)
    w = torch.randn(4, 5)
    tensors = [("conv1/weights", a, 1), ("conv1/weights/Adam", w, 1), ("global_step", g, 9)]
    data, entries, off = b"", [], 0
    for name, t, dt in tensors:
        raw = t.numpy().tobytes()
        entries.append((name.encode(), _spec_entry(dt, list(t.shape), off, len(raw), _mask(_crc32c(raw)))))
        data += raw
        off += len(raw)
    header = b"\x08\x01" + b"\x1a\x02\x08\x01"          # num_shards 1, version {producer 1}
    kv = [(b"", header)] + sorted(entries)
    prefix = str(tmp_path / "model.ckpt-12")
    open(prefix + ".index", "wb").write(_spec_table(kv))
    open(prefix + ".data-00000-of-00001", "wb").write(data)
    got = TB.read_bundle(prefix)
    assert sorted(got) == sorted(n for n, _, _ in tensors)
    for name, t, _ in tensors:
        assert got[name].dtype == t.dtype and torch.equal(got[name], t), name
    hdr, _ = TB.read_index(prefix)
    assert hdr["num_shards"] == 1 and hdr["producer"] == 1


def test_written_bundle_matches_the_spec(tmp_path):
    """Our writer's files decoded by the independent reader: keys sorted, header first, each
    entry's offset / size / masked crc32c describing the data shard."""
    tensors = {"softmax_linear/biases": torch.randn(29), "rnn/brnn-0/bidirectional_rnn/fw/GRUCell/W": torch.randn(3, 7),
               "global_step": torch.tensor(11, dtype=torch.int64), "x/bf16": torch.randn(5).bfloat16()}
    prefix = str(tmp_path / "model.ckpt-11")
    TB.write_bundle(prefix, tensors)
    kv = _spec_parse_table(open(prefix + ".index", "rb").read())
    assert kv[0][0] == b"" and [k for k, _ in kv[1:]] == sorted(k.encode() for k in tensors)
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    for k, v in kv[1:]:
        e = TB.decode_entry(v)
        t = tensors[k.decode()]
        raw = data[e["offset"]:e["offset"] + e["size"]]
        assert raw == t.view(torch.uint8).numpy().tobytes() if t.dtype == torch.bfloat16 else raw == t.numpy().tobytes()
        assert e["crc32c"] == _mask(_crc32c(raw)) and e["shape"] == tuple(t.shape) and e["dtype"] == t.dtype


def test_many_entries_span_blocks_and_roundtrip(tmp_path):
    """> 256 KiB of index entries (several data blocks through our writer), every dtype the
    reference's graph can hold, scalars and empty tensors."""
    tensors = {"v/%05d/%s" % (i, "x" * 40): torch.randn(3) for i in range(6000)}
    tensors.update({"i32": torch.arange(5, dtype=torch.int32), "f64": torch.randn(2, 2, dtype=torch.float64),
                    "b": torch.tensor([True, False]), "h": torch.randn(3).half(), "empty": torch.empty(0, 4),
                    "scalar": torch.tensor(2.5)})
    prefix = str(tmp_path / "p")
    TB.write_bundle(prefix, tensors, threads=4)
    assert os.path.getsize(prefix + ".index") > 256 * 1024
    got = TB.read_bundle(prefix)
    assert sorted(got) == sorted(tensors)
    for k, t in tensors.items():
        assert got[k].dtype == t.dtype and got[k].shape == t.shape and torch.equal(got[k], t), k


def test_sharded_bundle(tmp_path):
    """A big bundle goes out as several data shards written in parallel (TF's sharded Saver
    layout: the header counts them, each entry names its shard); the independent reader agrees."""
    tensors = {"w%d" % i: torch.randn(1000 + 37 * i) for i in range(10)}
    tensors["step"] = torch.tensor(3, dtype=torch.int64)
    prefix = str(tmp_path / "model.ckpt-3")
    TB.write_bundle(prefix, tensors, num_shards=3)
    files = sorted(os.listdir(tmp_path))
    assert files == ["model.ckpt-3.data-0000%d-of-00003" % i for i in range(3)] + ["model.ckpt-3.index"]
    kv = _spec_parse_table(open(prefix + ".index", "rb").read())
    hdr = TB.decode_header(kv[0][1])
    assert hdr["num_shards"] == 3
    shards = [open(TB.shard_name(prefix, i, 3), "rb").read() for i in range(3)]
    used = set()
    for k, v in kv[1:]:
        e = TB.decode_entry(v)
        used.add(e["shard_id"])
        raw = shards[e["shard_id"]][e["offset"]:e["offset"] + e["size"]]
        assert raw == tensors[k.decode()].numpy().tobytes() and e["crc32c"] == _mask(_crc32c(raw))
    assert used == {0, 1, 2}
    got = TB.read_bundle(prefix)
    for k, t in tensors.items():
        assert torch.equal(got[k], t)
    # rewriting the prefix with another shard count leaves no stale shard behind
    TB.write_bundle(prefix, tensors, num_shards=1)
    assert sorted(os.listdir(tmp_path)) == ["model.ckpt-3.data-00000-of-00001", "model.ckpt-3.index"]
    assert torch.equal(TB.read_bundle(prefix)["w9"], tensors["w9"])


def test_corruption_is_detected(tmp_path):
    prefix = str(tmp_path / "c")
    TB.write_bundle(prefix, {"a": torch.randn(100), "b": torch.randn(10)})
    d = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    d[5] ^= 0x40
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(d))
    with pytest.raises(ValueError, match="checksum"):
        TB.read_bundle(prefix)
    TB.read_bundle(prefix, verify=False)                  # readable when asked not to verify
    TB.write_bundle(prefix, {"a": torch.randn(100)})
    ix = bytearray(open(prefix + ".index", "rb").read())
    ix[3] ^= 0x01
    open(prefix + ".index", "wb").write(bytes(ix))
    with pytest.raises(RuntimeError, match="checksum"):
        TB.read_index(prefix)


def test_checkpoint_manager_writes_tf_names_and_restores(tmp_path):
    """The train driver's default format: TF variable names + Adam slots + EMA shadows +
    global_step / beta powers; restore() continues bitwise; an index whose global_step was
    written by TF semantics (next step) is honoured; a hand-written TF-only bundle (no
    deepspeech_amd/adam_t) recovers Adam's t from beta1_power."""
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    from deepspeech_amd.data.synthetic import FixedShapeBatches, to_device
    from deepspeech_amd.utils import checkpoint as CK
    torch.manual_seed(0)
    mk = lambda: Trainer(DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=2), LRSchedule(1e-3, 2, 0.5))  # noqa
    t = mk()
    b = to_device(FixedShapeBatches(2, max_frames=120, seed=0, pool=1).next(), torch.device("cpu"))
    for _ in range(4):
        t.step(b)
    CK.CheckpointManager(str(tmp_path), async_save=False).save(t, 3)
    raw = TB.read_bundle(str(tmp_path / "model.ckpt-3"))
    assert "rnn/brnn-1/bidirectional_rnn/bw/CustomRNNCell2/U/Adam_1" in raw
    assert "softmax_linear/weights/ExponentialMovingAverage" in raw
    assert int(raw["global_step"]) == 4 and int(raw[CK.ADAM_T]) == 4
    t2 = mk()
    assert CK.restore(t2, str(tmp_path)) == 3 and t2.global_step == 4 and t2.opt.t == 4
    for x, y in ((t.arena.flat, t2.arena.flat), (t.opt.m, t2.opt.m), (t.opt.v, t2.opt.v), (t.opt.ema, t2.opt.ema)):
        assert torch.equal(x, y)
    assert float(t.step(b)) == float(t2.step(b)) and torch.equal(t.arena.flat, t2.arena.flat)
    # a TF-written bundle carries no adam_t: recovered from beta1_power = 0.9^t
    del raw[CK.ADAM_T]
    TB.write_bundle(str(tmp_path / "tf" / "model.ckpt-3"), raw)
    t3 = mk()
    CK.restore(t3, str(tmp_path / "tf" / "model.ckpt-3"))
    assert t3.opt.t == 4 and t3.global_step == 4


@pytest.mark.parametrize("policy", ["abort", "skip"])
def test_nonfinite_loss_drops_saves_only_under_abort(tmp_path, policy):
    """a non-finite loss must not stop every later checkpoint under nan_policy skip
    (the skipped updates keep the weights finite); under abort the save is dropped and
    reported."""
    from deepspeech_amd.utils import checkpoint as CK

    class _T:
        def __init__(self, t):
            self.inner = t

        def __getattr__(self, k):
            return getattr(self.inner, k)

        def first_nonfinite_step(self):
            return 1
    from deepspeech_amd.models import DeepSpeech2
    from deepspeech_amd.trainer import LRSchedule, Trainer
    tr = _T(Trainer(DeepSpeech2(num_filters=4, num_hidden=16, num_rnn_layers=1), LRSchedule(1e-3, 2, 0.5)))
    m = CK.CheckpointManager(str(tmp_path), async_save=False, nan_policy=policy)
    path = m.save(tr, 3)
    if policy == "abort":
        assert path is None and m.dropped == [3] and CK.latest_checkpoint(str(tmp_path)) is None
    else:
        assert path is not None and m.written == [3] and TB.bundle_exists(path)
