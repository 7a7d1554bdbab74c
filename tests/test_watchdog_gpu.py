"""Failure detection for hipGraph-captured steps: a replay that outlives the
process-group timeout must abort the RCCL communicator and end the rank non-zero, and the ringdp
launcher must report the failure - the same contract as a hung eager collective.  One GPU, one
rank; the stall is a bounded spin kernel inside the graph."""
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = os.path.join(ROOT, "tests", "scripts", "graph_watchdog_script.py")


def _launch(stall_cycles: int, timeout_ms: int, split=None):
    env = dict(os.environ, WD_TIMEOUT_MS=str(timeout_ms))
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "ringdp.run", "--standalone", "--nproc-per-node", "1", SCRIPT,
                        str(stall_cycles)] + ([f"split={split}"] if split is not None else []), cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=120)
    return r, time.time() - t0


@pytest.mark.parametrize("split", [None, "1", ""])
def test_stalled_replay_is_aborted_by_watchdog(split):
    """~1-3 s of spinning (clock-rate dependent) against a 300 ms group timeout.  split: the segmented capture -
    "1": bucket 1 between segments (its eager collective's deadline or the replay beacon fires first), "":
    every collective inline, so only the replay beacon closing the last segment can see the stall."""
    r, dt = _launch(stall_cycles=3_000_000_000, timeout_ms=300, split=split)
    err = r.stderr
    if split == "1":
        assert "split plan ['inline', 'split', 'inline (last)']" in r.stdout, r.stdout
    elif split == "":
        assert "split plan ['inline', 'inline', 'inline (last)']" in r.stdout, r.stdout
    assert r.returncode != 0, (r.stdout, err[-3000:])
    assert "watchdog" in err, err[-3000:]
    if split != "1":
        assert "graph_replay" in err, err[-3000:]
    assert "failed with exit code" in err  # ringdp.run reported the dead rank


@pytest.mark.parametrize("split", [None, "1"])
def test_replay_within_timeout_is_not_flagged(split):
    r, dt = _launch(stall_cycles=1000, timeout_ms=60_000, split=split)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "replay finished" in r.stdout
