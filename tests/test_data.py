"""Native data runtime: CRC32C, TFRecord framing, tf.train.Example codec (checked against the protobuf library),
windowed/interleaved loader semantics, exact resume, text preparation, checkpoint blob IO."""
import gzip
import json
import os
import struct

import numpy as np
import pytest
import torch

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.data import native as N
from homebrewnlp_mtf_amd.data import pipeline as P
from homebrewnlp_mtf_amd.data import tfrecord as T


# ---------------------------------------------------------------------------------------------------------------
def test_crc32c_vectors():
    assert T.crc32c(b"123456789") == 0xE3069283
    assert T.crc32c(b"") == 0
    assert T.crc32c(bytes(32)) == 0x8A9136AA
    big = os.urandom(1 << 16)
    # incremental == one shot
    import ctypes
    L = N.lib()
    b = ctypes.create_string_buffer(big, len(big))
    c1 = L.rt_crc32c(ctypes.cast(b, ctypes.c_void_p), 1000, 0)
    c2 = L.rt_crc32c(ctypes.c_void_p(ctypes.addressof(b) + 1000), len(big) - 1000, c1)
    assert c2 == T.crc32c(big)


def _tf_example_classes():
    """tf.train.Example built from a hand-written descriptor (no TensorFlow here)"""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name="ex_test.proto", package="tftest", syntax="proto3")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for num, (fname, ftype, label, tname, packed) in enumerate(fields, 1):
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
            if packed:
                f.options.packed = True
        return m
    FD = descriptor_pb2.FieldDescriptorProto
    msg("BytesList", [("value", FD.TYPE_BYTES, FD.LABEL_REPEATED, None, False)])
    msg("FloatList", [("value", FD.TYPE_FLOAT, FD.LABEL_REPEATED, None, True)])
    msg("Int64List", [("value", FD.TYPE_INT64, FD.LABEL_REPEATED, None, True)])
    feat = fd.message_type.add(name="Feature")
    for i, (n, t) in enumerate([("bytes_list", ".tftest.BytesList"), ("float_list", ".tftest.FloatList"),
                                ("int64_list", ".tftest.Int64List")], 1):
        feat.field.add(name=n, number=i, type=FD.TYPE_MESSAGE, label=FD.LABEL_OPTIONAL, type_name=t, oneof_index=0)
    feat.oneof_decl.add(name="kind")
    feats = fd.message_type.add(name="Features")
    entry = feats.nested_type.add(name="FeatureEntry")
    entry.field.add(name="key", number=1, type=FD.TYPE_STRING, label=FD.LABEL_OPTIONAL)
    entry.field.add(name="value", number=2, type=FD.TYPE_MESSAGE, label=FD.LABEL_OPTIONAL, type_name=".tftest.Feature")
    entry.options.map_entry = True
    feats.field.add(name="feature", number=1, type=FD.TYPE_MESSAGE, label=FD.LABEL_REPEATED,
                    type_name=".tftest.Features.FeatureEntry")
    ex = fd.message_type.add(name="Example")
    ex.field.add(name="features", number=1, type=FD.TYPE_MESSAGE, label=FD.LABEL_OPTIONAL, type_name=".tftest.Features")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tftest.Example"))


def test_example_codec_matches_protobuf():
    Example = _tf_example_classes()
    toks = np.array([0, 1, 127, 128, 50256, 2 ** 40, -5], dtype=np.int64)
    raw = T.encode_example({"text": toks, "frame": [b"abc", b"", b"\x00\xff"], "f": np.array([1.5, -2.0],
                                                                                                dtype=np.float32)})
    m = Example()
    m.ParseFromString(raw)
    assert list(m.features.feature["text"].int64_list.value) == toks.tolist()
    assert list(m.features.feature["frame"].bytes_list.value) == [b"abc", b"", b"\x00\xff"]
    assert list(m.features.feature["f"].float_list.value) == [1.5, -2.0]
    # and the other direction: protobuf-serialised (incl. unpacked ints) decoded natively
    m2 = Example()
    m2.features.feature["text"].bytes_list.value.append("héllo €".encode())
    m2.features.feature["ids"].int64_list.value.extend([3, 4, 5])
    m2.features.feature["x"].float_list.value.extend([0.25])
    e = T.Example(m2.SerializeToString())
    assert e.bytes_list("text") == ["héllo €".encode()]
    assert e.int64("ids").tolist() == [3, 4, 5]
    assert e.float("x").tolist() == [0.25]
    assert e.text_tokens().tolist() == [ord(c) for c in "héllo €"]
    assert e.kind("missing") == (0, 0)


def test_utf8_decode_replacement():
    assert T.utf8_decode("aé€😀".encode()).tolist() == [97, 0xe9, 0x20ac, 0x1f600]
    assert T.utf8_decode(b"a\xffb\xc3").tolist() == [97, 0xfffd, 98, 0xfffd]
    assert T.utf8_decode(b"\xc0\xaf").tolist() == [0xfffd, 0xfffd]       # overlong


def test_tfrecord_roundtrip_and_corruption(tmp_path):
    path = str(tmp_path / "a.tfrecord")
    recs = [os.urandom(n) for n in (0, 1, 100, 70000)]
    with T.TFRecordWriter(path) as w:
        for r in recs:
            w.write(r)
    assert list(T.read_records(path)) == recs
    assert T.count_records(path) == 4
    # framing: u64 length + masked crc
    blob = open(path, "rb").read()
    assert struct.unpack("<Q", blob[:8])[0] == 0
    assert struct.unpack("<I", blob[8:12])[0] == T.crc32c(blob[:8], masked=True)
    bad = bytearray(blob)
    bad[-10] ^= 0xff
    open(path, "wb").write(bytes(bad))
    with pytest.raises(N.RuntimeErrorNative, match="crc"):
        list(T.read_records(path, verify_crc=True))
    assert len(list(T.read_records(path, verify_crc=False))) == 4


# ---------------------------------------------------------------------------------------------------------------
def _write_int64_file(path, records):
    with T.TFRecordWriter(path) as w:
        for r in records:
            w.write_example({"text": np.asarray(r, dtype=np.int64)})


def _py_windows(records, window, shift, skip=0):
    out = []
    toks_all = [np.asarray(r) for r in records]
    for toks in toks_all:
        if skip:
            d = min(skip, len(toks))
            toks, skip = toks[d:], skip - d
        k = 0
        while k * shift + window <= len(toks):
            out.append(toks[k * shift:k * shift + window])
            k += 1
    return out


def _py_interleave(per_file, cycle):
    """tf.data interleave(cycle_length, block_length=1)"""
    slots = [None] * cycle
    nxt, out, ci, n_open = 0, [], 0, 0
    while nxt < len(per_file) or n_open:
        if slots[ci] is not None:
            if slots[ci]:
                out.append(slots[ci].pop(0))
                ci = (ci + 1) % cycle
                continue
            slots[ci] = None
            n_open -= 1
            ci = (ci + 1) % cycle
        elif nxt < len(per_file):
            slots[ci] = list(per_file[nxt])
            nxt += 1
            n_open += 1
        else:
            ci = (ci + 1) % cycle
    return out


def _make_files(tmp_path, n_files=5, seed=0):
    rng = np.random.default_rng(seed)
    files, recs = [], []
    for i in range(n_files):
        rr = [rng.integers(0, 1000, int(rng.integers(5, 60))) for _ in range(int(rng.integers(1, 4)))]
        path = str(tmp_path / f"int64_test_{i:_>6d}_{sum(len(r) for r in rr)}.tfrecord")
        _write_int64_file(path, rr)
        files.append(path)
        recs.append(rr)
    return files, recs


@pytest.mark.parametrize("cycle", [1, 2, 3, 8])
def test_loader_window_interleave_semantics(tmp_path, cycle):
    files, recs = _make_files(tmp_path)
    window, shift = 9, 8
    expect = _py_interleave([_py_windows(r, window, shift) for r in recs], cycle)
    ld = P.TextLoader(files, window, shift, batch=1, cycle=cycle)
    got = [b[0].numpy() for b in ld]
    assert len(got) == len(expect)
    for g, e in zip(got, expect):
        assert g.tolist() == list(e)


def test_loader_batching_skip_and_repeat(tmp_path):
    files, recs = _make_files(tmp_path, 3)
    skips = [3, 0, 7]
    flat = _py_interleave([_py_windows(r, 5, 4, s) for r, s in zip(recs, skips)], 2)
    ld = P.TextLoader(files, 5, 4, batch=3, cycle=2, skips=skips)
    got = list(ld)
    assert len(got) == len(flat) // 3                 # remainder dropped
    assert torch.equal(torch.cat(got).view(-1, 5), torch.tensor(np.stack(flat[:len(got) * 3]), dtype=torch.int32))
    rep = P.TextLoader(files, 5, 4, batch=3, cycle=2, repeat=True)
    many = [rep.next()[1].clone() for _ in range(3 * len(flat))]
    assert len(many) == 3 * len(flat)


@pytest.mark.parametrize("shuffle,prefetch", [(0, 0), (0, 3), (16, 0), (16, 2)])
def test_loader_exact_resume(tmp_path, shuffle, prefetch):
    files, _ = _make_files(tmp_path, 6, seed=1)
    kw = dict(window=7, shift=6, batch=2, cycle=3, repeat=True, shuffle_buffer=shuffle, seed=5, prefetch=prefetch)

    def take(ld, n):
        out = []
        for _ in range(n):
            idx, t = ld.next()
            out.append(t.clone())
            ld.release(idx)
        return out

    a = P.TextLoader(files, **kw)
    take(a, 11)
    st = a.state()
    cont = take(a, 9)
    a.close()
    b = P.TextLoader(files, **kw)
    b.restore(st)
    again = take(b, 9)
    for x, y in zip(cont, again):
        assert torch.equal(x, y)
    # wrong file list is rejected
    c = P.TextLoader(files[:-1], **kw)
    with pytest.raises(N.RuntimeErrorNative):
        c.restore(st)


def test_loader_bytes_mode(tmp_path):
    path = str(tmp_path / "bytes_x_000000_1_20.tfrecord")
    text = "hello wörld, this is text"
    with T.TFRecordWriter(path) as w:
        w.write_example({"text": text.encode()})
    ld = P.TextLoader([path], 5, 4, batch=1)
    first = ld.next()[1]
    assert first[0].tolist() == [ord(c) for c in text[:5]]


def test_device_feeder_cpu(tmp_path):
    files, recs = _make_files(tmp_path, 4, seed=3)
    p = ModelParameter(dict(heads=1, features=4, use_video=False, sequence_length=8, token_patch_size=1,
                            output_offset=1, dataset_configs=[{"type": "text", "path": str(tmp_path / "*.tfrecord"),
                                                               "weight": 1}], interleaved_datasets=2,
                            shuffle_input_filenames=False))
    feeder = P.text_input(p, batch=2, dp_rank=0, dp_size=1, device="cpu", prefetch=2)
    b = feeder.next()
    assert b["token_x"].shape == (2, 8, 1) and b["token_y"].shape == (2, 8, 1)
    assert torch.equal(b["token_x"][:, 1:], b["token_y"][:, :-1])
    st = feeder.consumed_state
    nxt = feeder.next()
    feeder.close()
    feeder2 = P.text_input(p, batch=2, dp_rank=0, dp_size=1, device="cpu", prefetch=2, state=st)
    assert torch.equal(feeder2.next()["token_x"], nxt["token_x"])
    feeder2.close()


# ---------------------------------------------------------------------------------------------------------------
def test_split_files_sharding():
    files = [f"int64_x_{i:_>6d}_{100 + i}.tfrecord" for i in range(10)]
    a0, s0 = P.split_files(files, 0, 2, seed=456772)
    a1, s1 = P.split_files(files, 1, 2, seed=456772)
    assert sorted(a0 + a1) == sorted(files) and not set(a0) & set(a1)
    assert P.split_files(files, 0, 2, seed=456772) == (a0, s0)
    assert P.split_files(files, 0, 1, seed=0)[0] == sorted(files)


def test_simulate_data_pipeline_hand_case():
    # 2 files of 100 elements, ctx 10, patch 1: usable = 100 - ((100-1) % 10) - 1 = 90 → 9 windows each
    files = ["int64_a_000000_100.tfrecord", "int64_b_000001_100.tfrecord"]
    run = dict(steps=5, ctx=10, slice_count=1, interleave_size=2, batch_size=1, grad_accumulation=1,
               token_patch_size=1)
    depleted, used = P.simulate_data_pipeline([run], files)
    assert used == [30, 20] and depleted == [False, False]   # round robin a,b,a,b,a
    run["steps"] = 50
    depleted, used = P.simulate_data_pipeline([run], files)
    assert used == [90, 90] and depleted == [True, True]
    kept, skips = P.split_files(files, 0, 1, 0, [dict(run, steps=5)])
    assert kept == files and skips == [30, 20]


# ---------------------------------------------------------------------------------------------------------------
def _zstd_raw_frame(data: bytes) -> bytes:
    """a valid single-segment zstd frame holding one raw block (no compressor needed)"""
    assert len(data) < 256
    hdr = struct.pack("<I", 0xFD2FB528) + bytes([0x20, len(data)])
    blk = 1 | (0 << 1) | (len(data) << 3)
    return hdr + struct.pack("<I", blk)[:3] + data


def test_jsonl_to_text_and_tfrecords(tmp_path):
    import ctypes
    docs = [{"text": "line one\n    indented \"quoted\" \\ é", "meta": {"a": [1, 2, {"b": None}]}},
            {"meta": "x", "text": "emoji 😀 tab\t"}]
    raw = "\n".join(json.dumps(d) for d in docs) + "\n"
    L = N.lib()
    outs = []
    for name, blob in (("d.jsonl", raw.encode()), ("d.jsonl.gz", gzip.compress(raw.encode())),
                       ("d.jsonl.zst", _zstd_raw_frame(raw.encode()[:200]) if len(raw.encode()) < 200 else None)):
        if blob is None:
            continue
        src = tmp_path / name
        src.write_bytes(blob)
        dst = str(tmp_path / (name + ".txt"))
        stats = (ctypes.c_longlong * 2)()
        n = L.rt_jsonl_to_text(N.enc(str(src)), N.enc(dst), b"text", 4, 1, 0, stats)
        assert n == 2, N.last_error()
        outs.append(open(dst, "rb").read().decode())
    want = "".join(d["text"].replace("    ", "\t") + chr(4) for d in docs)
    assert all(o == want for o in outs)
    # text → bytes TFRecords in 16-byte chunks (cut on UTF-8 boundaries)
    txt = str(tmp_path / "d.jsonl.txt")
    n = L.rt_text_to_tfrecords(N.enc(txt), N.enc(str(tmp_path / "out_")), b"pile", 16, 0)
    assert n > 1
    names = sorted(f for f in os.listdir(tmp_path) if f.startswith("out_bytes_pile_"))
    assert len(names) == n and names[0].startswith("out_bytes_pile______0_")
    pieces = [T.Example(next(T.read_records(str(tmp_path / f)))).bytes_list("text")[0] for f in names]
    assert b"".join(pieces).decode() == want
    assert all(P._element_count(f) == len(pc) for f, pc in zip(names, pieces))


def test_zstd_frame_source(tmp_path):
    import ctypes
    raw = b'{"text": "zstd works"}\n'
    src = tmp_path / "a.jsonl.zst"
    src.write_bytes(_zstd_raw_frame(raw))
    dst = str(tmp_path / "a.txt")
    n = N.lib().rt_jsonl_to_text(N.enc(str(src)), N.enc(dst), b"text", -1, 0, 0, None)
    assert n == 1, N.last_error()
    assert open(dst).read() == "zstd works"


def test_blob_io_roundtrip_and_crc(tmp_path):
    from homebrewnlp_mtf_amd.utils import blobio
    arrs = [np.random.default_rng(0).standard_normal(n).astype(np.float32) for n in (1, 1000, 300000)]
    path = str(tmp_path / "shard.bin")
    meta = blobio.write_blobs(path, [a.view(np.uint8) for a in arrs])
    outs = [np.zeros_like(a) for a in arrs]
    blobio.read_blobs(path, [o.view(np.uint8) for o in outs], meta)
    for a, o in zip(arrs, outs):
        assert np.array_equal(a, o)
    with open(path, "r+b") as f:
        f.seek(meta["offsets"][2] + 12)
        f.write(b"\x01\x02")
    with pytest.raises(N.RuntimeErrorNative, match="CRC"):
        blobio.read_blobs(path, [o.view(np.uint8) for o in outs], meta)
