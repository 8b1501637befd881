"""CPU: host logic around the engine — parameter validation, device checks (the product path
refuses CPU tensors and has no CPU fallback), shard partitioning."""
import numpy as np
import pytest
import torch

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, sharding
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd._native import NativeLibraryError
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import risk_metrics
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams


def test_risk_params_validation():
    RiskParams().validate()
    with pytest.raises(ValueError):
        RiskParams(alpha=0.0).validate()
    with pytest.raises(ValueError):
        RiskParams(delta=float("inf")).validate()


def test_engine_refuses_cpu_tensors():
    s = torch.zeros((1, 2, 10, 2), dtype=torch.float64)
    with pytest.raises(ValueError, match="GPU"):
        engine.safe_halfspaces(s, torch.zeros((2, 2), dtype=torch.float64))


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback_without_gpu():
    with pytest.raises(NativeLibraryError):
        risk_metrics.device()
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import halfspaces
    with pytest.raises(NativeLibraryError):
        halfspaces.compute_safe_halfspaces([np.zeros((5, 2))], np.zeros(2), 0.3, 0.3, 0.2, 0.1, 0.15)


def test_risk_metric_kind():
    with pytest.raises(ValueError):
        risk_metrics.RiskMetric("var")
    assert risk_metrics.RiskMetric("cvar").params.alpha == 0.2


@pytest.mark.parametrize("units,world", [(0, 2), (1, 2), (7, 2), (200, 8), (1920, 8), (12800, 8), (5, 8)])
def test_shard_bounds_partition(units, world):
    spans = [sharding.shard_bounds(units, world, r) for r in range(world)]
    covered = []
    for a, b in spans:
        assert 0 <= a <= b <= units
        covered.extend(range(a, b))
    assert covered == list(range(units))
    per = -(-units // world) if units else 0
    assert all(b - a <= per for a, b in spans)


@pytest.mark.parametrize("O,T,world", [(3, 5, 4), (1, 7, 3), (4, 4, 2), (2, 3, 8), (5, 1, 2), (256, 50, 8)])
def test_shard_views_are_views_and_map_units(O, T, world):
    """Each rank's block is at most three strided views of the global tensor (never a copy, even
    for the reference's permuted [O, N, T, 2] order) and covers exactly units [start, stop)."""
    N = 3
    base = torch.arange(O * T * N * 2, dtype=torch.float64)
    layouts = [base.reshape(O, T, N, 2), base.reshape(O, N, T, 2).permute(0, 2, 1, 3)]
    ego = torch.arange(T * 2, dtype=torch.float64).reshape(T, 2)
    for s in layouts:
        seen = []
        for r in range(world):
            views, a, b = sharding.shard_views(s, ego, world, r)
            assert len(views) <= 3
            assert sum(c for *_, c in views) == b - a
            for sv, ev, off, cnt in views:
                assert sv.untyped_storage().data_ptr() == s.untyped_storage().data_ptr()
                o_n, t_n = sv.shape[:2]
                assert o_n * t_n == cnt and sv.shape[2:] == (N, 2)
                for k in range(cnt):
                    u = a + off + k
                    assert torch.equal(sv[k // t_n, k % t_n], s[u // T, u % T])
                    assert torch.equal(ev[k % t_n], ego[u % T])
                    seen.append(u)
        assert seen == list(range(O * T))


def test_shard_pieces_rejects_bad_blocks():
    with pytest.raises(ValueError):
        sharding.shard_pieces(2, 3, 4, 7)
    assert sharding.shard_pieces(2, 3, 2, 2) == []
    assert sharding.shard_pieces(4, 5, 3, 17) == [(0, 1, 3, 5, 0), (1, 3, 0, 5, 2), (3, 4, 0, 2, 12)]
