"""TensorBundle (tf.train.Saver format) writer/reader without TensorFlow: LevelDB table structure, protobuf field
encoding, CRCs, every dtype, and native checkpoint -> bundle -> trainer round trip. Parity with TF's own reader is
unpinned (no TensorFlow and no TF-written checkpoint in the reference tree); the wire rules are checked instead."""
import struct

import numpy as np
import torch

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.parallel import state as pstate
from homebrewnlp_mtf_amd.run.trainer import Trainer
from homebrewnlp_mtf_amd.utils import checkpoint as ckpt
from homebrewnlp_mtf_amd.utils import tensorbundle as TB

from test_runtime_cpu import CFG, _batch


def test_varint_and_entry_proto_encoding():
    assert TB._varint(0) == b"\x00" and TB._varint(300) == b"\xac\x02"
    # BundleHeaderProto{num_shards: 1, version{producer: 1}}
    assert TB.header_proto() == b"\x08\x01\x1a\x02\x08\x01"
    e = TB.entry_proto(1, [3, 0, 5], 128, 60, 0xdeadbeef)
    d = TB.decode_entry(e)
    assert d == {"dtype": 1, "shape": [3, 0, 5], "shard_id": 0, "offset": 128, "size": 60, "crc32c": 0xdeadbeef}
    assert e[-5:] == b"\x35" + struct.pack("<I", 0xdeadbeef)   # field 6, wire type 5 (fixed32)


def test_masked_crc_matches_leveldb_definition():
    # CRC32C("123456789") = 0xE3069283 (RFC 3720 check value); LevelDB mask: rot15 + 0xa282ead8
    crc = 0xE3069283
    want = (((crc >> 15) | (crc << 17)) + 0xa282ead8) & 0xFFFFFFFF
    assert TB.masked_crc32c(b"123456789") == want


def test_table_structure_many_blocks(tmp_path):
    items = [(f"var{i:05d}/slot".encode(), bytes([i % 251]) * (i % 97)) for i in range(2000)]
    path = str(tmp_path / "t.index")
    TB.write_table(path, items)
    raw = open(path, "rb").read()
    assert struct.unpack_from("<Q", raw, len(raw) - 8)[0] == 0xdb4775248b80fb57
    back = TB.read_table(path)
    assert back == sorted(items)
    # corrupting a data block byte must trip its CRC
    bad = bytearray(raw)
    bad[10] ^= 0xFF
    open(path, "wb").write(bytes(bad))
    try:
        TB.read_table(path)
        raise AssertionError("corruption not detected")
    except ValueError:
        pass


def test_bundle_round_trip_dtypes(tmp_path):
    torch.manual_seed(0)
    tensors = {"a/f32": torch.randn(3, 4), "b/bf16": torch.randn(5, 2).to(torch.bfloat16),
               "c/i64": np.arange(7, dtype=np.int64), "global_step": np.asarray(42, dtype=np.int64),
               "d/empty": np.zeros((0, 3), dtype=np.float32), "e/i32": np.array([[1, -2]], dtype=np.int32)}
    prefix = str(tmp_path / "model.ckpt-42")
    TB.write(prefix, tensors)
    back = TB.read(prefix)
    assert set(back) == set(tensors)
    assert np.array_equal(back["a/f32"], tensors["a/f32"].numpy())
    assert np.array_equal(back["b/bf16"], tensors["b/bf16"].float().numpy())
    assert back["global_step"].shape == () and int(back["global_step"]) == 42
    assert back["d/empty"].shape == (0, 3)
    entries = dict(TB.read_table(prefix + ".index"))
    assert TB.decode_entry(entries[b"b/bf16"])["dtype"] == TB.DT_BFLOAT16


def test_checkpoint_export_and_load(tmp_path):
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    a = Trainer(ModelParameter(CFG), "cpu")
    a.step(_batch(0))
    path = ckpt.save(a, str(tmp_path / "run"), 1, keep=1)
    n = TB.export_checkpoint(path, str(tmp_path / "export" / "model.ckpt-1"))
    back = TB.read(str(tmp_path / "export" / "model.ckpt-1"))
    assert len(back) == n and int(back["global_step"]) == 1
    assert any("/momentum" in k for k in back)          # optimizer slots travel with reference slot names
    torch.manual_seed(5)
    b = Trainer(ModelParameter(dict(CFG, seed=3)), "cpu")
    assert not torch.equal(a.store.master, b.store.master)
    step = TB.load_into(b, str(tmp_path / "export" / "model.ckpt-1"))
    assert step == 1 and torch.equal(a.store.master, b.store.master)
