"""CPU model of chain_kernel's hand-over between waves (csrc/kernels_wave.hip, round 4).

The kernel's exchange is pure index arithmetic -- blocks of kChainBlock wall ticks ending in
a barrier, wave w two blocks behind wave w - 1, ring slots at compile-time offsets from a
per-block base, writer stores in pairs in the unmasked blocks (components 1..K-1 only) and
lane 0 taking component 0 from the ring only at level 0.  This model replays exactly that
schedule (the same block, slot and masking rules, restated here) and checks, for every value
lane 0 of a wave consumes while it is at a level in [0, nsteps): the slot holds the upwind
wave's exit state of the previous chain tick, with the components used, written in an earlier
barrier block than the read and not overwritten before it.  A GPU run that caught a wrong
component 0 in round 4 (tests/test_wavefront_gpu.py, CN at 512 cells) is the reason it
exists: these rules are checked here on the CPU, over the geometries the kernel runs.
"""
import pytest

BLOCK, SKEW, RING = 8, 16, 32


def replay(nw, used, nsteps, K, level0_only=True):
    """Every read and write of every wave boundary, in the kernel's order; returns the
    failures (empty: the hand-over is exact).  level0_only=False restates round 4's first
    version, in which a masked tick took lane 0's component 0 from the ring at any level."""
    ticks = nsteps + used - 1
    nblocks = (ticks + (nw - 1) * SKEW + BLOCK - 1) // BLOCK
    writes = {}   # (region, slot) -> list of (block, tag, comps)
    reads = []    # (wave, block of the read, slot, consuming tick, components that matter)

    def unmasked_block(w, t0):
        u_lo = min(64 * w + 63, used - 1) + 1
        u_hi = max(u_lo, nsteps + 64 * w)
        return K > 1 and t0 >= u_lo and t0 + BLOCK <= u_hi

    for w in range(nw):
        wsk = w * SKEW
        writer = w < nw - 1
        for b in range(nblocks):
            t0 = b * BLOCK - wsk
            unmasked = unmasked_block(w, t0)
            for i in range(BLOCK):
                t = t0 + i
                if not unmasked and (t < 0 or t >= ticks):
                    continue
                # the prefetch of slot t + 1, consumed at tick t + 1 by lane 0
                tc = t + 1
                lvl = tc - 64 * w
                tc_block_t0 = (tc + wsk) // BLOCK * BLOCK - wsk
                need = set(range(1, K))
                if K == 1 or (not unmasked_block(w, tc_block_t0) and (lvl == 0 or not level0_only)):
                    need.add(0)
                if w > 0 and 0 <= lvl < nsteps:
                    reads.append((w, b, tc % RING, tc, frozenset(need)))
                if writer:
                    if unmasked:
                        if i & 1:
                            for tt in (t - 1, t):
                                writes.setdefault((w + 1, (tt + 1) % RING), []).append((b, tt, frozenset(range(1, K))))
                    else:
                        writes.setdefault((w + 1, (t + 1) % RING), []).append((b, t, frozenset(range(K))))
    fails = []
    for (w, br, slot, tick, need) in reads:
        hist = writes.get((w, slot), [])
        before = [x for x in hist if x[0] < br]
        if any(x[0] == br for x in hist):
            fails.append(("race in the read's block", w, tick, slot))
            continue
        if not before:
            fails.append(("never written", w, tick, slot))
            continue
        blk, tag, comps = before[-1]
        if tag != tick - 1:
            fails.append(("stale slot", w, tick, slot, tag))
        elif not need <= comps:
            fails.append(("component missing", w, tick, slot, sorted(need - comps)))
    return fails


@pytest.mark.parametrize("K", [1, 2, 5])
@pytest.mark.parametrize("nw,used", [(2, 65), (2, 128), (4, 200), (4, 256), (8, 449), (8, 512), (3, 150)])
@pytest.mark.parametrize("nsteps", [1, 7, 63, 64, 65, 150, 1000])
def test_chain_handover_exact(K, nw, used, nsteps):
    assert replay(nw, used, nsteps, K) == []


def test_model_catches_component_0_from_unmasked_writes():
    """The model is not vacuous: round 4's first rule (component 0 from the ring in every
    masked tick) fails in the geometry the GPU test caught (CN, 512 cells as 4 waves x 2
    cells per lane, 150 steps), on exactly 'component missing'."""
    bad = replay(4, 256, 150, 2, level0_only=False)
    assert bad and all(f[0] == "component missing" for f in bad)
