"""TensorFlow Saver-V2 checkpoint bundles without TensorFlow.

Reference: the reference trains with ``tf.train.Saver(tf.global_variables(), max_to_keep=100)``
and ``saver.save(sess, train_dir/model.ckpt, global_step=step)`` every 10 steps
(src/deepSpeech_train.py:354-356, :471), restores the latest through
``get_checkpoint_state`` (:383-398), and evaluates the EMA shadows restored from the same files
(src/deepSpeech_test.py:93-109, :217-220). Those files are a V2 *tensor bundle*:

  <prefix>.data-00000-of-00001   every tensor's raw little-endian bytes, back to back (a big
                                 bundle: .data-0000i-of-0000N shards, TF's sharded layout)
  <prefix>.index                 SSTable (LevelDB table format): "" -> BundleHeaderProto,
                                 variable name -> BundleEntryProto

This module encodes / decodes the two protobuf messages (hand-rolled wire format: they are a
handful of scalar fields) and drives the native parts in ``runtime/tensor_bundle.cpp``:
the SSTable codec, crc32c, and the shard writer that streams tensors straight from (pinned)
host memory with a pwrite per tensor on a thread pool, checksumming on the way.

  BundleHeaderProto { int32 num_shards = 1; Endianness endianness = 2; VersionDef version = 3; }
  BundleEntryProto  { DataType dtype = 1; TensorShapeProto shape = 2; int32 shard_id = 3;
                      int64 offset = 4; int64 size = 5; fixed32 crc32c = 6; repeated slices = 7; }
  TensorShapeProto  { repeated Dim dim = 2 { int64 size = 1; string name = 2; }; bool unknown_rank = 3; }
  VersionDef        { int32 producer = 1; int32 min_consumer = 2; repeated int32 bad_consumers = 3; }

Parity with TF-written files is unpinned: TensorFlow is not importable here and the reference
ships no checkpoint; the tests check round trips and an index assembled by hand from the format
description (tests/test_tf_bundle.py). Sliced (partitioned) variables and DT_STRING tensors are
not supported; the reference creates neither.
"""
from __future__ import annotations

import glob
import os
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

from ..runtime import native

DATA_SUFFIX = ".data-00000-of-00001"
INDEX_SUFFIX = ".index"
# a bundle of more than this many bytes is written as several data shards, each by its own
# thread: buffered writes to ONE file serialise on its inode lock (~5.5 GB/s per file measured on
# the MI355X boxes: 0.14 s for the headline's 0.74 GB), separate files do not
SHARD_BYTES = 96 << 20
MAX_SHARDS = 8


def shard_name(prefix: str, i: int, n: int) -> str:
    return "%s.data-%05d-of-%05d" % (prefix, i, n)

# tensorflow/core/framework/types.proto
_DT = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int16: 5, torch.int8: 6,
       torch.int64: 9, torch.bool: 10, torch.bfloat16: 14, torch.float16: 19}
_DT_INV = {v: k for k, v in _DT.items()}
_KTENSOR_BUNDLE_VERSION = 1


# ---- protobuf wire format ---------------------------------------------------------------------
def _varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3) + _varint(v)


def _field_bytes(num: int, b: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(b)) + b


def _field_fixed32(num: int, v: int) -> bytes:
    return _varint((num << 3) | 5) + int(v).to_bytes(4, "little")


def _parse(buf: bytes) -> Dict[int, list]:
    """Field number -> list of values (int for varint / fixed, bytes for length-delimited)."""
    out: Dict[int, list] = {}
    i, n = 0, len(buf)

    def rd_varint():
        nonlocal i
        r, shift = 0, 0
        while True:
            if i >= n or shift > 63:
                raise ValueError("bundle: truncated varint")
            b = buf[i]
            i += 1
            r |= (b & 0x7F) << shift
            if not b & 0x80:
                return r
            shift += 7
    while i < n:
        key = rd_varint()
        num, wt = key >> 3, key & 7
        if wt == 0:
            v = rd_varint()
        elif wt == 1:
            v = int.from_bytes(buf[i:i + 8], "little")
            i += 8
        elif wt == 2:
            ln = rd_varint()
            v = bytes(buf[i:i + ln])
            if len(v) != ln:
                raise ValueError("bundle: truncated field")
            i += ln
        elif wt == 5:
            v = int.from_bytes(buf[i:i + 4], "little")
            i += 4
        else:
            raise ValueError("bundle: unsupported wire type %d" % wt)
        out.setdefault(num, []).append(v)
    return out


def encode_header(num_shards: int = 1) -> bytes:
    return _field_varint(1, num_shards) + _field_bytes(3, _field_varint(1, _KTENSOR_BUNDLE_VERSION))


def encode_entry(dtype: torch.dtype, shape, offset: int, size: int, crc: int, shard: int = 0) -> bytes:
    dims = b"".join(_field_bytes(2, _field_varint(1, int(d))) for d in shape)
    msg = _field_varint(1, _DT[dtype]) + _field_bytes(2, dims)
    if shard:
        msg += _field_varint(3, shard)
    if offset:
        msg += _field_varint(4, offset)
    if size:
        msg += _field_varint(5, size)
    return msg + _field_fixed32(6, crc)


def decode_entry(buf: bytes) -> dict:
    f = _parse(buf)
    if 7 in f:
        raise ValueError("bundle: sliced (partitioned) variables are not supported")
    shape = []
    unknown = False
    if 2 in f:
        sp = _parse(f[2][0])
        unknown = bool(sp.get(3, [0])[0])
        for d in sp.get(2, []):
            shape.append(int(_parse(d).get(1, [0])[0]))
    if unknown:
        raise ValueError("bundle: tensor of unknown rank")
    dt = f.get(1, [0])[0]
    if dt not in _DT_INV:
        raise ValueError("bundle: unsupported dtype %d (DT_STRING and friends are not read)" % dt)
    return {"dtype": _DT_INV[dt], "shape": tuple(shape), "shard_id": f.get(3, [0])[0],
            "offset": f.get(4, [0])[0], "size": f.get(5, [0])[0], "crc32c": f.get(6, [None])[0]}


def decode_header(buf: bytes) -> dict:
    f = _parse(buf)
    ver = _parse(f[3][0]) if 3 in f else {}
    return {"num_shards": f.get(1, [1])[0], "endianness": f.get(2, [0])[0],
            "producer": ver.get(1, [0])[0], "min_consumer": ver.get(2, [0])[0]}


# ---- bundles ----------------------------------------------------------------------------------
def bundle_exists(prefix: str) -> bool:
    return os.path.exists(prefix + INDEX_SUFFIX)


def bundle_files(prefix: str) -> List[str]:
    return [prefix + INDEX_SUFFIX] + sorted(glob.glob(glob.escape(prefix) + ".data-*-of-*"))


def _host_bytes(t: torch.Tensor) -> Tuple[int, int, torch.Tensor]:
    """(address, nbytes, keep-alive) of a contiguous CPU copy of ``t`` (no copy when it is one)."""
    if t.device.type != "cpu":
        t = t.cpu()
    if not t.is_contiguous():
        t = t.contiguous()
    return t.data_ptr(), t.numel() * t.element_size(), t


def write_bundle(prefix: str, tensors: Dict[str, torch.Tensor], threads: int = 8,
                 num_shards: Optional[int] = None) -> None:
    """Write ``tensors`` (name -> CPU tensor; views of pinned buffers are written in place,
    without a copy) as a V2 bundle at ``prefix``. ``num_shards`` data files (default: one per
    SHARD_BYTES, at most MAX_SHARDS), balanced by bytes and written in parallel (TF's sharded
    Saver layout: each entry names its shard). The data shards are written first and the index
    last, each through a temporary name, so a reader never sees an index without its data."""
    N = native.load()
    names = sorted(tensors)
    for n in names:
        if n == "" or tensors[n].dtype not in _DT:
            raise ValueError("bundle: cannot store %r (%s)" % (n, tensors[n].dtype))
    keep, ptrs, sizes = {}, {}, {}
    for n in names:
        p, nb, k = _host_bytes(tensors[n].detach())
        keep[n], ptrs[n], sizes[n] = k, p, nb
    total = sum(sizes.values())
    ns = num_shards or max(1, min(MAX_SHARDS, -(-total // SHARD_BYTES)))
    ns = max(1, min(ns, len(names) or 1))
    # greedy balance: largest tensors first, each to the lightest shard
    shard_of, load = {}, [0] * ns
    for n in sorted(names, key=lambda x: -sizes[x]):
        i = min(range(ns), key=lambda j: load[j])
        shard_of[n] = i
        load[i] += sizes[n]
    members = [[n for n in names if shard_of[n] == i] for i in range(ns)]
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    per = max(1, int(threads) // ns)

    def write(i):
        return N.bundle_write_shard(shard_name(prefix, i, ns) + ".tmp", [ptrs[n] for n in members[i]],
                                    [sizes[n] for n in members[i]], per)
    if ns == 1:
        crc_lists = [write(0)]
    else:
        with ThreadPoolExecutor(max_workers=ns) as ex:
            crc_lists = list(ex.map(write, range(ns)))
    where = {}
    for i in range(ns):
        off = 0
        for n, c in zip(members[i], crc_lists[i]):
            where[n] = (i, off, c)
            off += sizes[n]
    items = [(b"", encode_header(ns))]
    for n in names:
        i, off, c = where[n]
        items.append((n.encode(), encode_entry(keep[n].dtype, keep[n].shape, off, sizes[n], c, shard=i)))
    tmp_index = prefix + INDEX_SUFFIX + ".tmp"
    N.bundle_write_file(tmp_index, N.bundle_build_table(items))
    for old in glob.glob(glob.escape(prefix) + ".data-*-of-*"):
        if not old.endswith(".tmp"):
            os.remove(old)                       # a previous bundle at this prefix
    for i in range(ns):
        os.replace(shard_name(prefix, i, ns) + ".tmp", shard_name(prefix, i, ns))
    os.replace(tmp_index, prefix + INDEX_SUFFIX)


def read_index(prefix: str, verify: bool = True) -> Tuple[dict, Dict[str, dict]]:
    """(header, name -> entry) of the bundle at ``prefix``."""
    with open(prefix + INDEX_SUFFIX, "rb") as f:
        kv = native.load().bundle_parse_table(f.read(), verify)
    header, entries = None, {}
    for k, v in kv:
        if k == b"":
            header = decode_header(v)
        else:
            entries[k.decode()] = decode_entry(v)
    if header is None:
        raise ValueError("bundle %s: index has no header entry" % prefix)
    if header["endianness"] != 0:
        raise ValueError("bundle %s: big-endian bundles are not supported" % prefix)
    if header["num_shards"] < 1:
        raise ValueError("bundle %s: bad shard count %d" % (prefix, header["num_shards"]))
    return header, entries


def read_bundle(prefix: str, names: Optional[Iterable[str]] = None, verify: bool = True) -> Dict[str, torch.Tensor]:
    """name -> CPU tensor of every (or the named) variable of the bundle at ``prefix``; with
    ``verify`` each tensor's bytes are checked against the index's crc32c."""
    header, entries = read_index(prefix, verify)
    want = list(entries) if names is None else list(names)
    N = native.load()
    ns = header["num_shards"]
    maps = {}

    def shard(i):
        if i not in maps:
            path = shard_name(prefix, i, ns)
            maps[i] = np.memmap(path, dtype=np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)
        return maps[i]
    out = {}
    for n in want:
        e = entries[n]
        nb = int(e["size"])
        if not 0 <= e["shard_id"] < ns:
            raise ValueError("bundle %s: %s names shard %d of %d" % (prefix, n, e["shard_id"], ns))
        data = shard(e["shard_id"])
        raw = np.array(data[e["offset"]:e["offset"] + nb])          # a private copy off the map
        if raw.size != nb:
            raise ValueError("bundle %s: %s lies beyond the data shard" % (prefix, n))
        if verify and e["crc32c"] is not None and N.bundle_masked_crc32c(raw) != e["crc32c"]:
            raise ValueError("bundle %s: checksum mismatch for %s" % (prefix, n))
        t = torch.from_numpy(raw).view(e["dtype"]) if nb else torch.empty(0, dtype=e["dtype"])
        out[n] = t.reshape(e["shape"])
    maps.clear()
    return out
