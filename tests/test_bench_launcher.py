"""bench.py's rank plumbing on CPU (no GPU, no HIP call): `--gpus N` without a launcher starts N
child ranks itself, a launcher's WORLD_SIZE that disagrees with --gpus is refused, and a rank
that dies takes the whole run down with a non-zero exit (the reference only ever
picks one GPU, train_e2v.py:3-14)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
sys.path.insert(0, ROOT)

LAUNCH_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
               "TORCHELASTIC_RUN_ID", "V2E2V_RANK_LAUNCHER", "V2E2V_DRY_FAIL_RANK")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_KEYS}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_gpus_2_launches_two_ranks_one_line():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "3"], _env())
    assert r.returncode == 0, r.stderr
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["ranks_seen"] == 2 and ln["process_group"] == "gloo"
    assert len(set(ln["rank_pids"])) == 2               # two processes, neither of them the parent


def test_gpus_1_stays_single_process():
    r = _run(["--gpus", "1", "--dry-run", "--steps", "2"], _env())
    assert r.returncode == 0, r.stderr
    (ln,) = _json_lines(r.stdout)
    assert ln["n_gpus"] == 1 and ln["ranks_seen"] == 1 and ln["process_group"] is None


def test_launcher_world_size_mismatch_refused():
    env = _env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT="29512",
               TORCHELASTIC_RUN_ID="t")
    r = _run(["--gpus", "8", "--dry-run"], env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and not _json_lines(r.stdout)


def test_failed_rank_fails_the_run():
    r = _run(["--gpus", "2", "--dry-run"], _env(V2E2V_DRY_FAIL_RANK="1"), timeout=240)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)


def test_rank_plan(monkeypatch):
    import argparse
    import bench
    for k in LAUNCH_KEYS:
        monkeypatch.delenv(k, raising=False)
    ns = lambda g: argparse.Namespace(gpus=g)            # noqa: E731
    assert bench.rank_plan(ns(None)) == ("single", 1)
    assert bench.rank_plan(ns(1)) == ("single", 1)
    assert bench.rank_plan(ns(4)) == ("launch", 4)
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "x")
    a = ns(None)
    assert bench.rank_plan(a) == ("rank", 4) and a.gpus == 4     # torchrun without --gpus
    assert bench.rank_plan(ns(4)) == ("rank", 4)
    with pytest.raises(SystemExit):
        bench.rank_plan(ns(8))
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit):
        bench.rank_plan(ns(8))                                    # torchrun N=1 with --gpus 8


def test_terminated_launcher_stops_its_ranks():
    """SIGTERM to the launching process reaches every rank (forwarded, and PR_SET_PDEATHSIG if the
    launcher dies outright): no rank is left running -- on the GPU box, holding a GPU."""
    import signal
    import time
    psutil = pytest.importorskip("psutil")
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "400000000"],
                         env=_env(), cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        kids = []
        for _ in range(120):                          # the ranks are up once both are children
            kids = psutil.Process(p.pid).children()
            if len(kids) == 2:
                break
            time.sleep(0.25)
        assert len(kids) == 2
        time.sleep(2.0)
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) != 0
        gone, alive = psutil.wait_procs(kids, timeout=60)
        assert not alive
    finally:
        if p.poll() is None:
            p.kill()
