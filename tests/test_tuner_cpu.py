"""Fused-GEMM layout tuner rules (ops.tune_fused_splits), with the device
timing replaced by a synthetic cost model: the co-scheduling cap, the
fewest-workgroup fallback for shapes no layout fits under the cap (70B), the
short-tile fallback for the 8B Mpad-64 decode steps, and the env pin."""
import pytest

from loqa_hub_amd import ops


@pytest.fixture
def fake_timing(monkeypatch):
    """graph_time(fn) -> cost of the candidate that ``fn`` launches."""
    seen = []

    def graph_time(fn, reps=8, trials=3):
        fn()
        return seen[-1][1]

    monkeypatch.setattr(ops, "graph_time", graph_time)
    monkeypatch.setattr(ops, "_FSPLITS", {})
    return seen


def _tune(seen, key, cost, **kw):
    def run(s, rt, wr, i):
        seen.append(((s, rt, wr), cost(s, rt, wr)))
    return ops.tune_fused_splits(key, run, key[2], **kw)


def test_cap_excludes_faster_wide_grids(fake_timing):
    # 8B o projection: 4096 rows. split-K 2 with 16-row tiles (512 WGs) is
    # "fastest" in isolation but exceeds the 256-WG cap
    cost = lambda s, rt, wr: {(2, 1, 1): 1.0}.get((s, rt, wr), 2.0 + s + rt)
    best = _tune(fake_timing, ("resid", 4096, 4096, 16), cost, rts=(1, 2), wr4=True)
    units = (4096 // (16 * best[1] * best[2])) * best[0]
    assert units <= 256 and best != (2, 1, 1)
    tried = {c for c, _ in fake_timing}
    assert (2, 1, 1) not in tried


def test_fewest_workgroups_fallback(fake_timing):
    # 70B gate|up: 57344 rows, nothing fits under 256 WGs; the fewest-WG
    # layouts (4 waves along rows, 32-row tiles: 448 WGs) are the candidates
    cost = lambda s, rt, wr: 1.0 if (s, rt, wr) == (1, 2, 4) else 3.0
    best = _tune(fake_timing, ("silu", 57344, 8192, 16), cost, rts=(1, 2), wr4=True)
    assert best == (1, 2, 4)
    tried = {c for c, _ in fake_timing}
    assert all((57344 // (16 * rt * wr)) * s <= 2 * 448 for s, rt, wr in tried)


def test_short_tile_fallback_without_fewest(fake_timing):
    # 8B gate|up at Mpad 64 beside the Whisper decoder: no wide layouts; the
    # first candidate (16-row tiles, no split) is taken without timing others
    cost = lambda s, rt, wr: 5.0
    best = _tune(fake_timing, ("silu", 28672, 4096, 64), cost, rts=(1, 2), wr4=False, fewest=False)
    assert best == (1, 1, 1)


def test_env_pin_overrides(fake_timing, monkeypatch):
    monkeypatch.setenv("LOQA_FSPLIT_OVERRIDE", "resid:4096x14336:M16=2,2,1;silu:1x1:M16=1,1,1")
    best = _tune(fake_timing, ("resid", 4096, 14336, 16), lambda *a: 1.0, rts=(1, 2))
    assert best == (2, 2, 1) and not fake_timing


def test_decode_cap_context(fake_timing):
    cost = lambda s, rt, wr: 1.0 / ((4096 // (16 * rt * wr)) * s)    # more WGs = faster
    with ops.decode_cap(128):
        best = _tune(fake_timing, ("resid", 4096, 4096, 32), cost, rts=(1, 2), wr4=True)
    assert (4096 // (16 * best[1] * best[2])) * best[0] <= 128
