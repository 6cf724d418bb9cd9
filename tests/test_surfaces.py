"""Host-side trainer surfaces the reference scripts touch (no GPU needed)."""
import pytest
import torch


def test_stable_trainer_optimizer_scheduler_criterion():
    """StableTrainer keeps the reference's .optimizer / .scheduler / .criterion (mc:229-240): Adam(lr, wd 1e-5,
    eps 1e-8), StepLR(step_size=15, gamma=0.7) stepped once per epoch, nn.BCELoss; param_groups[0]['lr'] is the
    live rate (read every epoch by the reference's driver, mc:414)."""
    from vad_amd.mc import SimpleVideoAnomalyDetector, StableTrainer
    m = SimpleVideoAnomalyDetector()
    tr = StableTrainer(m, [], [], "cpu", lr=1e-3)
    g = tr.optimizer.param_groups[0]
    assert g["lr"] == pytest.approx(1e-3) and g["weight_decay"] == 1e-5 and g["eps"] == 1e-8
    assert isinstance(tr.criterion, torch.nn.BCELoss)
    ref_opt = torch.optim.Adam(torch.nn.Linear(2, 2).parameters(), lr=1e-3)
    ref_sched = torch.optim.lr_scheduler.StepLR(ref_opt, step_size=15, gamma=0.7)
    for _ in range(40):
        tr.scheduler.step()
        ref_opt.step()
        ref_sched.step()
        assert tr.optimizer.param_groups[0]["lr"] == pytest.approx(ref_opt.param_groups[0]["lr"], rel=1e-12)
        assert tr._lr() == tr.optimizer.param_groups[0]["lr"]
    tr.optimizer.param_groups[0]["lr"] = 5e-4  # a user override is what the next device step uses
    assert tr._lr() == 5e-4
