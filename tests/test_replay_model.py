"""The link model that scripts/one_rank_of_p.py adds to a measured
one-rank-of-P replay (profiles/dist_rbt_replay_r6.md): per block the small
message's latency + transfer, and the column rest only where it is longer
than two chain steps (csrc/hip/drbt_exec.hip ships it two steps ahead of
its first use)."""
import importlib.util
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def orp():
    spec = importlib.util.spec_from_file_location("one_rank_of_p", ROOT / "scripts" / "one_rank_of_p.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_free_links_add_nothing(orp):
    m = orp.model(8192, 8, 7e-3, 0.7e-3, 0.2e-3, 2, lat_us=0.0, bw_gbs=1e12, t_chain_step=110e-6)
    assert m["link_factor_ms"] == pytest.approx(0.0, abs=1e-6)
    assert m["total_ms"] == pytest.approx(7.0 + 3 * (0.7 + 0.2), rel=1e-6)


def test_latency_counts_once_per_block_and_super_block(orp):
    # 8192 on 8 ranks: 63 small messages on the chain, 8 super-blocks x 2 directions x 3 applies
    a = orp.model(8192, 8, 7e-3, 0.7e-3, 0.2e-3, 2, lat_us=10.0, bw_gbs=1e12, t_chain_step=110e-6)
    assert a["link_factor_ms"] == pytest.approx(63 * 10e-3, rel=1e-6)
    assert a["solve_link_ms"] == pytest.approx(2 * 8 * 10e-3, rel=1e-6)


def test_rest_costs_only_beyond_two_chain_steps(orp):
    # with a short chain step the 8 MB rest at 50 GB/s (~160 us) is exposed at the top of the matrix
    slow = orp.model(8192, 8, 7e-3, 0.7e-3, 0.2e-3, 2, lat_us=0.0, bw_gbs=50.0, t_chain_step=20e-6)
    fast = orp.model(8192, 8, 7e-3, 0.7e-3, 0.2e-3, 2, lat_us=0.0, bw_gbs=50.0, t_chain_step=110e-6)
    small_only = sum(min(2 * 128, 8192 - k * 128) * 128 * 8 / 50e9 for k in range(1, 64)) * 1e3
    assert fast["link_factor_ms"] == pytest.approx(small_only, rel=1e-9)
    assert slow["link_factor_ms"] > fast["link_factor_ms"]
