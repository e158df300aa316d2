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


WORD_VTT = """WEBVTT
Kind: captions
Language: en

00:00:00.000 --> 00:00:02.000 align:start position:0%
hello<00:00:00.500><c> big</c><00:00:01.000><c> world</c>

00:00:02.000 --> 00:00:04.000 align:start position:0%
again<00:00:02.600><c> and</c><00:00:03.100><c> more</c>
"""

CUE_VTT = """WEBVTT

1
00:00:01.000 --> 00:00:03.000
one two
three four

2
00:00:03.000 --> 00:00:04.000
five
"""


def test_decode_vtt_word_timed_and_cues():
    import video2tfrecord as V2
    text, words, stamps = V2.decode_vtt(WORD_VTT)
    # each piece is stamped with the inline stamp that closes it; the line's last word runs into the next line
    # text after the last stamp joins the last group
    assert words == [" hello", " big", " world again", " and more"] and stamps == [0.5, 1.0, 2.6, 3.1]
    assert text == "".join(words)
    text, words, stamps = V2.decode_vtt(CUE_VTT)
    assert words == [" one", " two", " three", " four", " five"]       # cue numbers are not caption text
    assert stamps == [1.0, 1.5, 2.0, 2.5, 3.0] and text == " one two three four five"


def test_split_equal_balances_longest_first():
    import video2tfrecord as V2
    ids, dur = V2.split_equal(list("abcdef"), [900, 800, 300, 700, 100, 260], 2)
    assert ids == [["a", "c", "f"], ["b", "d"]] and dur == [[900, 300, 260], [800, 700]]   # e (100) is too short
    ids, _ = V2.split_equal(list("ab"), [1, 2], 3, min_duration=0)
    assert ids == [["b"], ["a"], []]


def test_word_split_encoders():
    import video2tfrecord as V2
    words = [" hello", " big", " world again"]
    enc = V2._Tokenizer(None)            # byte-level: one token per byte
    groups = V2.bpe_with_word_split(enc, words, "".join(words))
    # a token that is only spaces matches anywhere, so the group before takes it (BPE merges the space into the
    # next word's token, byte-level tokens keep it separate)
    assert [bytes(g).decode() for g in groups] == [" hello ", "big ", "world again"]
    assert V2.char_level_encoder([" hi"]) == [[32, 104, 105]]


def test_video2tfrecord_subtitles_and_text_only_frames(tmp_path):
    """a .vtt next to the video: words reach the frame whose window they end in; overflow beyond
    language_token_per_frame - 1 tokens goes to text-only skip_frame frames; a separator frame joins two videos"""
    pytest.importorskip("PIL")
    import video2tfrecord as V2
    rng = np.random.default_rng(1)
    for k in range(2):
        np.save(tmp_path / f"v{k}.npy", rng.integers(0, 256, (4, 8, 16, 3), dtype=np.uint8))
        (tmp_path / f"v{k}.vtt").write_text(CUE_VTT)
    out = tmp_path / "tfr"
    # 4 frames at 1 fps: windows end at 1, 2, 3, 4 s
    assert V2.main(["--out", str(out), "--name", "s", "--width", "16", "--height", "8", "--subtitles",
                    "--encoder", "char", "--fps", "1", "--language-token-per-frame", "4", "--padding-token", "0",
                    "--concat-token", "7", str(tmp_path / "v0.npy"), str(tmp_path / "v1.npy")]) == 0
    (f,) = [str(out / n) for n in os.listdir(out)]
    exs = [T.Example(r) for r in T.read_records(f)]
    rows = [(e.int64("skip_frame")[0], e.int64("concat")[0], e.int64("mask")[0],
             bytes(int(t) for t in e.int64("tokens")[:e.int64("mask")[0]] if 0 < int(t) < 256)) for e in exs]
    half = rows[:len(rows) // 2]
    # frame 0 (window 0-1 s): nothing stamped before 1.0; frame 1 (-2 s): " one" " two" = 8 chars -> 3 + 3 + 2
    assert half[0] == (0, 0, 0, b"")
    assert [r[3] for r in half[1:4]] == [b" on", b"e t", b"wo"] and [r[0] for r in half[1:4]] == [0, 1, 1]
    sep = rows[len(rows) // 2]
    assert sep[:3] == (0, 1, 4) and list(exs[len(rows) // 2].int64("tokens")) == [7, 7, 7, 7]
    assert rows[len(rows) // 2 + 1:] == half


def test_comm_probe_gloo_world2():
    """tools/comm_probe.py: bus-bandwidth rows for every collective over a 2-rank gloo group"""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OBST_DIST_BACKEND="gloo", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", "29517", os.path.join(root, "tools", "comm_probe.py"),
                        "--sizes-mb", "0.25,1", "--iters", "2", "--warmup", "1", "--dtype", "float32"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert {x["op"] for x in rows} == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}
    assert len(rows) == 8 and all(x["busbw_GBps"] > 0 and x["world"] == 2 for x in rows)
