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
