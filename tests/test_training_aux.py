"""Training auxiliaries: progressive layer drop schedule, curriculum schedules + sampler,
random-LTD, Hessian eigenvalue, MoQ fake quantization."""
import numpy as np
import pytest
import torch


def test_pld_schedule():
    from shuffle_exchange_amd.runtime.progressive_layer_drop import ProgressiveLayerDrop
    p = ProgressiveLayerDrop(theta=0.5, gamma=0.01)
    p.update_state(0)
    assert p.get_theta() == pytest.approx(1.0)
    p.update_state(10000)
    assert p.get_theta() == pytest.approx(0.5, abs=1e-6)
    assert p.get_state()["progressive_layer_drop"]


def test_curriculum_schedules():
    from shuffle_exchange_amd.runtime.data_pipeline import CurriculumScheduler
    lin = CurriculumScheduler({"min_difficulty": 8, "max_difficulty": 64, "schedule_type": "fixed_linear",
                               "schedule_config": {"total_curriculum_step": 100, "difficulty_step": 8}})
    vals = [lin.update_difficulty(s) for s in (1, 50, 100, 200)]
    assert vals[0] == 8 and vals[1] == 32 and vals[2] == 64 and vals[3] == 64
    disc = CurriculumScheduler({"min_difficulty": 1, "max_difficulty": 3, "schedule_type": "fixed_discrete",
                                "schedule_config": {"difficulty": [1, 2, 3], "max_step": [5, 10]}})
    assert [disc.get_difficulty(s) for s in (1, 6, 11)] == [1, 2, 3]


def test_curriculum_sampler_respects_threshold():
    from shuffle_exchange_amd.runtime.data_pipeline import CurriculumDataSampler, CurriculumScheduler
    metric = np.arange(1000) % 100
    sch = CurriculumScheduler({"min_difficulty": 10, "max_difficulty": 100, "schedule_type": "fixed_linear",
                               "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 10}})
    s0 = CurriculumDataSampler(metric, sch, global_batch_size=32, dp_rank=0, dp_size=2)
    b = s0.next_batch()
    assert len(b) == 16 and max(metric[b]) <= sch.get_current_difficulty()


def test_random_ltd_keeps_dropped_tokens():
    from shuffle_exchange_amd.runtime.data_pipeline import RandomLayerTokenDrop
    lin = torch.nn.Linear(8, 8)
    ltd = RandomLayerTokenDrop(lin)
    ltd.reserved_length = 3
    x = torch.randn(2, 10, 8)
    y = ltd(x)
    changed = (y != x).any(-1)
    assert changed.sum(1).tolist() == [3, 3]
    ltd.eval()
    assert torch.allclose(ltd(x), lin(x))


def test_eigenvalue_quadratic():
    from shuffle_exchange_amd.runtime.eigenvalue import Eigenvalue
    w = torch.nn.Parameter(torch.zeros(3))
    A = torch.diag(torch.tensor([1.0, 5.0, 2.0]))
    mod = torch.nn.Module()
    mod.w = w
    ev = Eigenvalue(max_iter=200, tol=1e-6)
    res = ev.compute_eigenvalue(mod, lambda: 0.5 * w @ A @ w)
    assert res[0][0] == pytest.approx(5.0, rel=1e-3)


def test_moq_fake_quantize():
    from shuffle_exchange_amd.runtime.quantize import Quantizer, fake_quantize
    w = torch.randn(16, 64)
    q = fake_quantize(w, 4, groups=4)
    assert len(torch.unique(q[:4])) <= 16
    qz = Quantizer(q_groups=4, q_start_bits=8, q_target_bits=4, q_period=1)
    p = torch.nn.Parameter(w.clone())
    for _ in range(6):
        qz.quantize([[p]])
    assert qz.bits[(0, 0)] == 4
