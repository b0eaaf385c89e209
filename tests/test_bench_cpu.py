"""CPU tier: bench.py's host logic that needs no GPU -- the watchdog's naming of the stalled rank
from the ranks' published progress.  The end-to-end stall rehearsal over
torch.distributed.run is tests/test_gpu_dist.py::test_bench_stalled_rank_exits_with_the_phase_named.
"""
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)


@pytest.fixture
def wd_env(tmp_path, monkeypatch):
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    monkeypatch.setenv("MASTER_PORT", "4711")
    import bench
    return bench


def _write(wd, rank, phase, seq, calls):
    with open(wd.paths[rank], "w") as fh:
        json.dump({"rank": rank, "phase": phase, "seq": seq, "in_phase_s": 12.0,
                   "collectives": calls}, fh)


def test_fewest_collectives_is_the_stalled_rank(wd_env):
    wd = wd_env.Watchdog(0, 3)
    # ranks 0 and 1 entered the first halo exchange of the phase; rank 2 never did
    for r, calls in ((0, 13), (1, 13), (2, 12)):
        _write(wd, r, "first applies", 7, calls)
    stalled, states = wd.stalled_ranks()
    assert stalled == [2] and sorted(states) == [0, 1, 2]


def test_equal_collectives_fall_back_to_the_earliest_phase(wd_env):
    wd = wd_env.Watchdog(1, 2)
    _write(wd, 0, "operator build", 2, -1)   # (no context attached yet)
    _write(wd, 1, "first applies", 7, -1)
    assert wd.stalled_ranks()[0] == [0]


def test_a_rank_without_state_never_started(wd_env):
    wd = wd_env.Watchdog(0, 4)
    for r in (0, 1, 3):
        _write(wd, r, "timed applies", 9, 40)
    assert wd.stalled_ranks()[0] == [2]


def test_no_difference_is_undetermined(wd_env):
    wd = wd_env.Watchdog(0, 2)
    for r in (0, 1):
        _write(wd, r, "timed gmres", 8, 100)
    assert wd.stalled_ranks()[0] == []


def test_state_files_are_per_job_and_removed_when_done(wd_env, tmp_path):
    wd = wd_env.Watchdog(1, 2)
    wd.phase("operator build", 60)  # publishes rank 1's state
    assert os.path.exists(wd.paths[1])
    assert all(str(tmp_path) in p and "_4711_" in p for p in wd.paths)
    wd.done()
    assert not os.path.exists(wd.paths[1])
