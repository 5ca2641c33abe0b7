"""The single-pass chain kernels' early tile hand-off as a checked invariant
(tools/isa_count.py --check-handoff, run by __graft_entry__.build()).

A producer raises its tile's flag after `s_waitcnt vmcnt(N)`, N = TS/4 (or 8)
outstanding stores, and that orders the flag after the tile's end-state stores
only if at least N vector-memory instructions follow those stores on every
path to the wait (csrc/chain_tile.hip, tile_cascade step 4-5).  These tests
run the check on synthetic listings (a store removed, a store behind a branch
that can skip it, a flag with no wait) and on the real gfx950 listing of
csrc/chain_tile.hip, as built and with one y store deleted by hand.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_count  # noqa: E402

LISTING = os.path.join(ROOT, "dsp-audio-project_amd", "build", "chain_tile.s")


def _prog(body):
    return isa_count._program(body.strip().split("\n"))


GOOD = """
	global_store_dwordx2 v50, v[58:59], s[4:5] sc1
	global_store_dwordx2 v50, v[60:61], s[4:5] offset:8 sc1
	s_and_saveexec_b64 s[2:3], vcc
	s_cbranch_execz .LBB0_41
	ds_write_b128 v74, v[42:45]
.LBB0_41:
	s_or_b64 exec, exec, s[2:3]
	buffer_store_dwordx4 v[80:83], v78, s[4:7], 0 offen nt
	buffer_store_dwordx4 v[84:87], v78, s[4:7], 0 offen offset:1024 nt
	buffer_store_dwordx4 v[88:91], v1, s[4:7], 0 offen nt
	buffer_store_dwordx4 v[92:95], v1, s[4:7], 0 offen offset:1024 nt
	s_cbranch_vccnz .LBB0_43
	s_waitcnt vmcnt(4)
	v_cmp_eq_u32_e32 vcc, 56, v0
.LBB0_43:
	global_store_dword v1, v2, s[4:5] sc1
	s_endpgm
"""


def test_counted_wait_synthetic():
    ins, labels = _prog(GOOD)
    assert isa_count.check_counted_wait(ins, labels) == [(4, 4)]
    # one y store fewer: the flag may overtake the state
    ins, labels = _prog(GOOD.replace(
        "\tbuffer_store_dwordx4 v[92:95], v1, s[4:7], 0 offen offset:1024 nt\n", "", 1))
    assert isa_count.check_counted_wait(ins, labels) == [(4, 3)]
    # a store the wave can branch around does not count
    skip = GOOD.replace("\tbuffer_store_dwordx4 v[88:91]",
                        "\ts_cbranch_scc1 .LBB0_9\n\tbuffer_store_dwordx4 v[88:91]").replace(
        "\tbuffer_store_dwordx4 v[92:95]", ".LBB0_9:\n\tbuffer_store_dwordx4 v[92:95]")
    ins, labels = _prog(skip)
    assert isa_count.check_counted_wait(ins, labels) == [(4, 3)]
    # a flag store with no wait behind the state stores
    ins, labels = _prog(GOOD.replace("\ts_waitcnt vmcnt(4)\n", ""))
    assert isa_count.check_counted_wait(ins, labels) == [(-1, 0)]


@pytest.fixture(scope="module")
def listing():
    if not os.path.exists(LISTING):
        subprocess.run(["make", "-C", os.path.join(ROOT, "dsp-audio-project_amd", "csrc"),
                        "../build/chain_tile.s"], check=True, capture_output=True)
    with open(LISTING) as f:
        return f.read()


def test_real_listing_passes_and_a_removed_store_fails(listing):
    seen, bad, report = isa_count.check_handoff(LISTING, listing)
    assert not bad, bad
    assert seen >= 6 and len(report) >= 6
    # delete the last y store before the first counted wait of k_chain_tile
    m = re.search(r"^(_Z\w*k_chain_tileI\w*):", listing, re.M)   # (not k_chain_tile3)
    body_start = m.start()
    wait = re.compile(r"^\s+s_waitcnt vmcnt\(([1-9]\d*)\)", re.M)
    states = [s.start() for s in re.finditer(r"^\s+global_store_dwordx2\b.*\bsc1\b", listing, re.M)
              if s.start() > body_start]
    w = next(x for x in wait.finditer(listing, states[0]))
    stores = [s for s in re.finditer(r"^\s+buffer_store_dwordx4\b.*\n", listing, re.M)
              if states[0] < s.start() < w.start()]
    assert len(stores) >= int(w.group(1))
    cut = stores[-1]
    edited = listing[:cut.start()] + listing[cut.end():]
    _, bad, _ = isa_count.check_handoff(LISTING, edited)
    assert any("counted hand-off wait" in b for b in bad), bad
