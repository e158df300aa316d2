"""Ops tools: watchdog restart logic, sweep expansion, text → TFRecord preparation and tokenizer training."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import run_experiments  # noqa: E402
import run_manager  # noqa: E402
import text2tfrecord  # noqa: E402

from homebrewnlp_mtf_amd.data import tfrecord as T  # noqa: E402
from homebrewnlp_mtf_amd.data import pipeline as P  # noqa: E402


def test_run_manager_restarts_failed_job(tmp_path):
    marker = tmp_path / "ran_once"
    script = f"import os,sys; p={str(marker)!r}\nif not os.path.exists(p): open(p,'w').close(); sys.exit(3)\nprint('ok')"
    rc = run_manager.run([sys.executable, "-c", script], log_path=str(tmp_path / "log"), poll=0.05)
    assert rc == 0
    log = open(tmp_path / "log").read()
    assert "exit status 3" in log and "ok" in log


def test_run_manager_kills_stalled_job(tmp_path):
    hb = tmp_path / "hb"
    count = tmp_path / "count"
    # first launch: never writes a heartbeat and sleeps (stall); second launch exits cleanly
    script = (f"import os,time; c={str(count)!r}; n=int(open(c).read()) if os.path.exists(c) else 0\n"
              f"open(c,'w').write(str(n+1))\n"
              f"if n == 0: time.sleep(60)\n")
    rc = run_manager.run([sys.executable, "-c", script], log_path=str(tmp_path / "log"),
                         heartbeat_glob=str(hb) + "*", stall_seconds=1.0, poll=0.1, startup_grace=0.0, grace=1.0)
    assert rc == 0 and open(count).read() == "2"
    assert "no heartbeat" in open(tmp_path / "log").read()


def test_run_manager_gives_up(tmp_path):
    rc = run_manager.run([sys.executable, "-c", "import sys; sys.exit(1)"], poll=0.05, max_restarts=2)
    assert rc == 1


def test_sweep_expansion(tmp_path):
    base = tmp_path / "base.json"
    base.write_text(json.dumps({"depth": 2, "learning_rate": 0.1}))
    grid = tmp_path / "grid.json"
    grid.write_text(json.dumps({"depth": [2, 4], "learning_rate": [0.1, 0.01, 0.001]}))
    names = list(run_experiments.expand(json.load(open(base)), json.load(open(grid)), 2))
    assert len(names) == 12 and len({n for n, _ in names}) == 12
    assert names[0][0] == "depth=2-learning_rate=0.1-run=0"
    rc = run_experiments.main(["--base-config", str(base), "--run-config", str(grid), "--prefix",
                               str(tmp_path / "runs") + "/", "--config-dir", str(tmp_path / "cfg"), "--dry-run"])
    assert rc == 0 and len(os.listdir(tmp_path / "cfg")) == 6


def test_text_prep_bytes_and_int64(tmp_path):
    docs = [{"text": f"document {i}: " + "lorem ipsum dolor sit amet " * (i + 3)} for i in range(20)]
    src = tmp_path / "a.jsonl"
    src.write_text("\n".join(json.dumps(d) for d in docs) + "\n")
    text2tfrecord.prep([str(src)], str(tmp_path / "txt"), procs=1)
    txt = str(tmp_path / "txt" / "0.txt")
    assert open(txt).read().count(chr(4)) == 20
    n = text2tfrecord.to_bytes([txt], str(tmp_path / "b"), "demo", 512)
    files = sorted(os.listdir(tmp_path / "b"), key=lambda f: int(f[len("bytes_demo_"):].lstrip("_").split("_")[0]))
    assert len(files) == n and all(f.startswith("bytes_demo_") for f in files)
    # the loader reads them back as code points
    ld = P.TextLoader([str(tmp_path / "b" / f) for f in files], 33, 32, batch=1, cycle=1)
    first = ld.next()[1][0].tolist()
    assert "".join(chr(c) for c in first) == open(txt).read()[:33]
    pytest.importorskip("tokenizers")
    import train_tokenizer
    tok = train_tokenizer.train([txt], str(tmp_path / "tok.json"), vocab_size=300)
    m = text2tfrecord.to_int64([txt], str(tmp_path / "i"), "demo", str(tmp_path / "tok.json"), 700)
    files = sorted(os.listdir(tmp_path / "i"), key=lambda f: int(f[len("int64_demo_"):].lstrip("_").split("_")[0]))
    assert len(files) == m and files[0].startswith("int64_demo______0_")
    ids = np.concatenate([T.Example(next(T.read_records(str(tmp_path / "i" / f)))).int64("text") for f in files])
    assert tok.decode(ids.tolist(), skip_special_tokens=False).replace(" ", "")[:40] == open(txt).read().replace(" ", "")[:40]
    assert all(P._element_count(f) == len(T.Example(next(T.read_records(str(tmp_path / "i" / f)))).int64("text"))
               for f in files)


def test_video_json_split_and_chunk(tmp_path):
    import video_json
    src = tmp_path / "v.json"
    src.write_text(json.dumps({"id": list(range(10)), "duration": [100, 5, 300, 50, 70, 20, 400, 10, 60, 90]}))
    ids, dur = video_json.split_equal([[i] for i in range(10)], [100, 5, 300, 50, 70, 20, 400, 10, 60, 90], 3, -1)
    sums = [sum(d) for d in dur]
    assert sum(sums) == 1105 and max(sums) - min(sums) <= 100
    assert sorted(i for part in ids for (i,) in part) == list(range(10))
    ci, cd = video_json.chunk(list(range(10)), [100, 5, 300, 50, 70, 20, 400, 10, 60, 90], 200)
    assert sorted(i for c in ci for i in c) == list(range(10))
    assert all(sum(d) >= 200 for d in cd[:-1])
    assert video_json.main(["split", str(src), "2", "--prefix", str(tmp_path) + "/"]) == 0
    assert (tmp_path / "work_split_1.json").exists()


def test_video2tfrecord_and_jannet_loader(tmp_path):
    pytest.importorskip("PIL")
    import torch
    import video2tfrecord
    from homebrewnlp_mtf_amd.config import ModelParameter
    from homebrewnlp_mtf_amd.data import video as V
    rng = np.random.default_rng(0)
    vids = []
    for k in range(2):
        arr = rng.integers(0, 256, (7, 8, 16, 3), dtype=np.uint8)
        path = tmp_path / f"v{k}.npy"
        np.save(path, arr)
        vids.append(str(path))
    texts = {"v0.npy": ["hi"] * 7, "v1.npy": ["there", "x"]}
    (tmp_path / "t.json").write_text(json.dumps(texts))
    out = tmp_path / "tfr"
    assert video2tfrecord.main(["--out", str(out), "--name", "demo", "--width", "16", "--height", "8",
                                "--text", str(tmp_path / "t.json"), "--language-token-per-frame", "4",
                                "--videos-per-file", "1"] + vids) == 0
    files = sorted(str(out / f) for f in os.listdir(out))
    assert len(files) == 2
    ex = T.Example(next(T.read_records(files[0])))
    assert ex.int64("tokens").tolist() == [104, 105, 0, 0] and ex.int64("mask").tolist() == [2]
    p = ModelParameter(dict(model_mode="jannet", use_video=True, use_language=True, heads=2, features_per_head=8,
                            sequence_length=2, time_patch=1, frame_width=16, frame_height=8, patch_size=4,
                            color_channels=3, three_axes=False, language_token_per_frame=4, token_patch_size=1,
                            vocab_size=256, experts=4, interleaved_datasets=2))
    src = V.VideoSource(files, p, batch=2, device="cpu", workers=2)
    b = src.next()
    assert b["frame"].shape == (2, 3, 8, 48) and b["frame"].dtype == torch.uint8
    assert b["token_x"].shape == (2, 2, 4, 1) and b["vid_msk_src"].all()
    # the first window of file 0 decodes back to the (JPEG-approximate) patches of frame 0
    ref = V.decode_frame(video2tfrecord.encode_jpeg(np.load(vids[0])[0], 16, 8), p)
    assert np.array_equal(b["frame"][0, 0].numpy(), ref)
    st = src.consumed_state
    nxt = src.next()
    src2 = V.VideoSource(files, p, batch=2, device="cpu", workers=2)
    src2.restore(st)
    assert torch.equal(src2.next()["frame"], nxt["frame"])
