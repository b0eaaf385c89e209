"""CPU tier: the ISA checker of the sweep's hand-counted LDS-DMA waits (tools/
check_sweep_waitcnt.py) on synthetic instruction streams -- it must flag an LDS read that a
DMA may not have written yet, on straight-line code and across branches and loops, and accept
one behind a wait that retires the DMA."""
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_sweep_waitcnt as C  # noqa: E402


def _scan(tmp_path, body):
    p = tmp_path / "k.s"
    p.write_text("kern:\n" + "\n".join("\t" + ln if not ln.startswith(".LBB") else ln
                                        for ln in body) + "\n.Lfunc_end0:\n")
    return C.scan(str(p))[2]


def test_uncovered_read_is_flagged(tmp_path):
    assert _scan(tmp_path, ["global_load_lds_dwordx4 v1, s[2:3]", "global_load_dwordx4 v[4:7], v1",
                            "s_waitcnt vmcnt(2)", "ds_read_b128 v[8:11], v2"])


def test_wait_retiring_the_dma_covers_the_read(tmp_path):
    assert not _scan(tmp_path, ["global_load_lds_dwordx4 v1, s[2:3]",
                                "global_load_dwordx4 v[4:7], v1", "global_load_dwordx4 v[8:11], v1",
                                "s_waitcnt vmcnt(2)", "ds_read_b128 v[8:11], v2"])


def test_worst_path_through_a_branch_is_flagged(tmp_path):
    # one path waits, the other jumps over the wait to the read
    assert _scan(tmp_path, ["global_load_lds_dwordx4 v1, s[2:3]", "s_cbranch_scc1 .LBB0_2",
                            ".LBB0_1:", "s_waitcnt vmcnt(0)", ".LBB0_2:",
                            "ds_read_b128 v[8:11], v2", "s_endpgm"])


def test_loop_carried_dma_is_flagged(tmp_path):
    # the DMA at the loop's end is outstanding at the read on the next trip
    assert _scan(tmp_path, ["s_waitcnt vmcnt(0)", ".LBB0_1:", "ds_read_b128 v[8:11], v2",
                            "global_load_lds_dwordx4 v1, s[2:3]", "s_cbranch_scc1 .LBB0_1",
                            "s_endpgm"])
