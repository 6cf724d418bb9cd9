"""CPU: the direct classifier's loss-mode upstream gradient is affine in the causal score c (csrc/mlp.hip dir_mid_kernel,
the seed rows of the forward-time precompute): d total / d logits = A + c * beta, with A, beta computed from the
logits and labels only.  Checked in float64 against autograd through the reference loss (cad:669-686 via
oracle.cad_oracle.cad_losses' composition), and the stacked-row backward of a gated MLP chain against the backward
of the combined rows (the linearity the precompute relies on)."""
import numpy as np
import torch
import torch.nn.functional as F


def seed_rows(logits: np.ndarray, labels: np.ndarray):
    """Mirror of dir_mid_kernel's seed: (A, beta) rows of d total / d logits = A + c beta."""
    B = logits.shape[0]
    mx = logits.max(axis=1, keepdims=True)
    e = np.exp(logits - mx)
    p = e / e.sum(axis=1, keepdims=True)
    q = np.exp(p - p.max(axis=1, keepdims=True))
    q = q / q.sum(axis=1, keepdims=True)
    onehot = np.eye(2)[labels]
    k = 0.4 * (0.3 * 2.0 / B)
    dpA = 0.4 * (q - onehot) / B
    dpA[:, 1] += k * (0.4 * p[:, 1] - labels)
    dpB = np.zeros_like(dpA)
    dpB[:, 1] = k * 0.6
    A = p * (dpA - (p * dpA).sum(axis=1, keepdims=True))
    beta = p * (dpB - (p * dpB).sum(axis=1, keepdims=True))
    return A, beta


def autograd_dlogits(logits, c, labels, kl):
    lg = torch.tensor(logits, dtype=torch.float64, requires_grad=True)
    cc = torch.tensor(c, dtype=torch.float64)
    y = torch.tensor(labels)
    yf = y.double()
    direct = torch.softmax(lg, dim=-1)
    final = 0.6 * cc + 0.4 * direct[:, 1]
    cls = F.cross_entropy(direct, y)
    anom = F.mse_loss(final, yf)
    causal = F.mse_loss(cc, yf)
    total = 0.4 * cls + 0.3 * anom + 0.2 * causal + 0.1 * torch.tensor(kl, dtype=torch.float64).mean()
    total.backward()
    return lg.grad.numpy()


def test_loss_grad_is_affine_in_causal_score():
    rng = np.random.default_rng(3)
    for B in (1, 2, 8):
        for _ in range(5):
            logits = rng.normal(size=(B, 2)) * 2
            c = rng.uniform(0, 1, size=B)
            labels = rng.integers(0, 2, size=B)
            kl = rng.normal(size=B)
            A, beta = seed_rows(logits, labels)
            ref = autograd_dlogits(logits, c, labels, kl)
            np.testing.assert_allclose(A + c[:, None] * beta, ref, rtol=1e-12, atol=1e-15)


def test_stacked_rows_backward_folds_to_the_combined_backward():
    """Input-gradient chain of the direct classifier's layers 4 .. 0 (ReLU / dropout gates of the forward rows) on the
    stacked rows [A; beta] then folded with c equals the chain on the rows A + c beta."""
    g = torch.Generator().manual_seed(0)
    B = 8
    widths = [6144, 512, 256, 128, 64, 2]
    Ws = [torch.randn(widths[i + 1], widths[i], generator=g, dtype=torch.float64) * 0.05 for i in range(5)]
    gates = [torch.randn(B, widths[i], generator=g, dtype=torch.float64) for i in range(1, 5)]  # h[i-1] > 0 masks
    gs = [1 / 0.7, 1 / 0.8, 1.0, 1.0]
    A = torch.randn(B, 2, generator=g, dtype=torch.float64)
    beta = torch.randn(B, 2, generator=g, dtype=torch.float64)
    c = torch.rand(B, generator=g, dtype=torch.float64)

    def chain(d, rows_gate):
        for i in range(4, 0, -1):
            d = (d @ Ws[i]) * (rows_gate(i - 1) > 0) * gs[i - 1]
        return d @ Ws[0]

    stacked = chain(torch.cat([A, beta]), lambda j: torch.cat([gates[j], gates[j]]))
    folded = stacked[:B] + c[:, None] * stacked[B:]
    direct = chain(A + c[:, None] * beta, lambda j: gates[j])
    torch.testing.assert_close(folded, direct, rtol=1e-12, atol=1e-12)
