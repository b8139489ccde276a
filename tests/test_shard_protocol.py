"""The sharded TermSearch protocol, checked on the CPU with the oracle.

A url-hash shard joins only its own rows, but every decision the reference takes
on container sizes -- J1 list existence, the J2 fold order and the J3 dispatch
of every step, including the size of the intermediate container -- must be the
one the single container takes (AbstractIndex.java:108-127,
ReferenceContainer.java:334-366,406-416).  libyrwi exchanges the global sizes
(yrwi_host.cpp plan_batch / run_join_phase); oracle/shard_fold.py restates that
protocol.  Planning each shard on its own sizes (round 1) flips dispatches near
the by-test threshold and is not bit-exact: the test keeps a count of those
flips so the corpus demonstrably covers the flip band."""

import numpy as np
import pytest

import oracle as orc
import shard_fold as sf
from yacy_search_server_amd import synth

NOW = 20741 * 86400000 + 12345


def _cat(parts):
    parts = [np.asarray(p, dtype=np.uint8).reshape(-1, 40) for p in parts]
    return np.concatenate(parts) if parts else np.zeros((0, 40), np.uint8)


@pytest.fixture(scope="module")
def small():
    full = synth.preset("small")
    return full, synth.build_index(full).as_dict()


@pytest.mark.parametrize("world", [2, 8])
def test_global_protocol_bit_exact_local_is_not(small, world):
    full, whole = small
    parts = [synth.build_index(full.shard(r, world)).as_dict() for r in range(world)]
    flips = 0
    for nex in (0, 1, 2):
        for inc, exc in synth.queries(full, 300, 2, 3, nex, qseed=7 + nex):
            ih = [synth.term_hash(full, t) for t in inc]
            eh = [synth.term_hash(full, t) for t in exc]
            ref = orc.term_search(whole, ih, eh, 2147483647, NOW)
            got = _cat(sf.sharded_term_search(parts, ih, eh, 2147483647, NOW, "global"))
            assert got.shape == ref.shape and np.array_equal(got, ref), (inc, exc)
            loc = _cat(sf.sharded_term_search(parts, ih, eh, 2147483647, NOW, "local"))
            flips += not (loc.shape == ref.shape and np.array_equal(loc, ref))
    assert flips > 0  # the query set reaches the dispatch flip band


def test_exclude_term_absent_from_a_shard(small):
    """A missing exclude term disables ALL exclusion (J1) -- globally, not per shard."""
    full, whole = small
    world = 8
    parts = [synth.build_index(full.shard(r, world)).as_dict() for r in range(world)]
    sizes = synth.counts(full)
    hashes = [synth.term_hash(full, t) for t in range(full.n_terms)]
    big = [int(t) for t in np.argsort(-sizes)[:3]]
    ih = [hashes[big[0]], hashes[big[1]]]
    # an exclude term with postings on shard 3 only: every 3rd url of that shard's
    # part of the include pair's first list
    rare = b"rareTERMxxxA"
    rows = parts[3][ih[0]][::3].copy()
    whole = dict(whole)
    whole[rare] = rows
    parts[3] = dict(parts[3])
    parts[3][rare] = rows
    hashes = hashes + [rare]
    rare = len(hashes) - 1
    for eh in ([hashes[rare], hashes[big[2]]], [hashes[rare]]):
        ref = orc.term_search(whole, ih, eh, 2147483647, NOW)
        got = _cat(sf.sharded_term_search(parts, ih, eh, 2147483647, NOW, "global"))
        assert np.array_equal(got, ref)
    # and a globally missing exclude term disables the other one everywhere
    missing = b"AAAAAAAAAAAA"
    ref = orc.term_search(whole, ih, [missing, hashes[big[2]]], 2147483647, NOW)
    assert len(ref) == len(orc.term_search(whole, ih, [], 2147483647, NOW))
    got = _cat(sf.sharded_term_search(parts, ih, [missing, hashes[big[2]]], 2147483647, NOW, "global"))
    assert np.array_equal(got, ref)
