"""Algorithmic work of one fused learner step, used by
bench.py for the roofline / MFMA-utilisation accounting."""


def flops_per_step(S, A, H1, H2, B, tf_recompute=False, survey=False):
    """FLOP of one fused learner step (ddpg.py:86-113) at batch B.

    Default (minimal) count, MAC per sample:
      3*AF (target fwd, online fwd, weight grads) + 4*CF (target fwd, train fwd,
      weight grads, action-grad fwd) + critic dX (H2 + 2*H1*H2)
      + action-grad dX (H2 + H1*H2 + A*H1; only the action half of dcat is
      needed) + actor dX (H2*A + H1*H2) + dQ head (H2).
    survey=True is SURVEY.md §8(d)'s count, which charges the full 2*H1*H2 for
    the action-grad dX; tf_recompute adds the reference's second actor forward."""
    AF = S * H1 + H1 * H2 + H2 * A
    CF = S * H1 + A * H1 + 2 * H1 * H2 + H2
    if survey:
        dX = 2 * (H2 + 2 * H1 * H2) + A * H1 + H2 * A + H1 * H2
    else:
        dX = 3 * H2 + 4 * H1 * H2 + A * H1 + H2 * A
    mac = 3 * AF + 4 * CF + dX
    if tf_recompute:
        mac += AF
    return 2 * B * mac
