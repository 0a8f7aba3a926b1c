"""Hypothesis-driven shape sweep of the TF-semantics oracle (SURVEY.md §4.2 "unit, CPU":
odd sizes, C=1/3, rectangular inputs, kernel/stride variants). Every property is checked
against an independent formulation: a direct loop for the SAME conv, the adjoint identity
for conv2d_transpose, a float64 two-pass formula for the moments, and TF's closed form for
Adam (Appendix A)."""
import math

import torch
from hypothesis import given, settings, strategies as st

from distributed_tensorflow_for_dcgan_amd.models.config import same_out, same_pads
from distributed_tensorflow_for_dcgan_amd.ops import reference as R

from test_reference_ops import naive_conv_same

SET = settings(max_examples=25, deadline=None)
_OLD = []


def setup_module(_):
    _OLD.append(torch.get_default_dtype())
    torch.set_default_dtype(torch.float64)


def teardown_module(_):
    torch.set_default_dtype(_OLD.pop())


def _gen(seed):
    return torch.Generator().manual_seed(seed)


@SET
@given(n=st.integers(1, 40), k=st.sampled_from([1, 3, 5]), s=st.sampled_from([1, 2, 3]))
def test_same_pads_properties(n, k, s):
    lo, hi = same_pads(n, k, s)
    out = same_out(n, s)
    assert out == math.ceil(n / s)
    assert lo + hi == max((out - 1) * s + k - n, 0)
    assert hi - lo in (0, 1)  # TF puts the odd pixel at the END (bottom/right)


@SET
@given(h=st.integers(2, 11), w=st.integers(2, 11), ci=st.sampled_from([1, 2, 3]), co=st.integers(1, 4),
       b=st.integers(1, 2), seed=st.integers(0, 2 ** 16))
def test_conv2d_same_rectangular_matches_loop(h, w, ci, co, b, seed):
    g = _gen(seed)
    x = torch.randn(b, h, w, ci, generator=g, dtype=torch.float64)
    wt = torch.randn(5, 5, ci, co, generator=g, dtype=torch.float64)
    y = R.conv2d_same(x, wt)
    assert y.shape == (b, same_out(h), same_out(w), co)
    assert torch.allclose(y, naive_conv_same(x, wt), atol=1e-9)


@SET
@given(hi=st.integers(1, 9), ci=st.sampled_from([1, 3, 4]), co=st.sampled_from([1, 3, 5]), odd=st.booleans(),
       seed=st.integers(0, 2 ** 16))
def test_conv_transpose_adjoint_any_size(hi, ci, co, odd, seed):
    """<conv(y), x> == <y, conv_T(x)> for every output size whose SAME conv maps back to hi."""
    ho = 2 * hi - 1 if (odd and hi > 1) else 2 * hi
    assert same_out(ho) == hi
    g = _gen(seed)
    x = torch.randn(2, hi, hi, co, generator=g, dtype=torch.float64)
    y = torch.randn(2, ho, ho, ci, generator=g, dtype=torch.float64)
    w = torch.randn(5, 5, ci, co, generator=g, dtype=torch.float64)       # conv: ci -> co
    lhs = (R.conv2d_same(y, w) * x).sum()
    rhs = (y * R.conv2d_transpose_same(x, w, (ho, ho))).sum()  # deconv layout [kh,kw,out,in]
    assert torch.allclose(lhs, rhs, rtol=1e-10, atol=1e-9)


@SET
@given(rows=st.integers(1, 64), c=st.integers(1, 8), groups=st.sampled_from([1, 2]), seed=st.integers(0, 2 ** 16))
def test_moments_are_biased_and_per_group(rows, c, groups, seed):
    x = torch.randn(groups * rows, 1, 1, c, generator=_gen(seed), dtype=torch.float64) * 3 + 1
    mean, var = R.moments(x, groups=groups)
    xs = x.reshape(groups, rows, c)
    m_ref = xs.mean(1)
    v_ref = ((xs - m_ref[:, None]) ** 2).mean(1)  # biased (divide by N, not N-1)
    assert torch.allclose(mean.reshape(groups, c), m_ref, atol=1e-12)
    assert torch.allclose(var.reshape(groups, c), v_ref, atol=1e-12)


@SET
@given(t=st.integers(1, 50), g=st.floats(-1e3, 1e3, allow_nan=False, allow_infinity=False),
       lr=st.sampled_from([2e-4, 1e-3]), b1=st.sampled_from([0.5, 0.9]))
def test_tf_adam_closed_form(t, g, lr, b1):
    """After t identical gradients g, TF-Adam's step equals the closed form with epsilon
    OUTSIDE the bias correction: lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps)."""
    b2, eps = 0.999, 1e-8
    p = torch.zeros(1, dtype=torch.float64)
    m = torch.zeros(1, dtype=torch.float64)
    v = torch.zeros(1, dtype=torch.float64)
    grad = torch.full((1,), g, dtype=torch.float64)
    prev = p.clone()
    for k in range(1, t + 1):
        prev = p.clone()
        R.tf_adam_update(p, grad, m, v, b1 ** k, b2 ** k, lr, b1, b2, eps)
    mt = (1 - b1 ** t) * g
    vt = (1 - b2 ** t) * g * g
    step = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t) * mt / (math.sqrt(vt) + eps)
    assert math.isclose(float(prev - p), step, rel_tol=1e-9, abs_tol=1e-15)


@SET
@given(x=st.lists(st.floats(-80, 80, allow_nan=False), min_size=1, max_size=16), t=st.sampled_from([0.0, 1.0]))
def test_bce_with_logits_stable_and_exact(x, t):
    lg = torch.tensor(x, dtype=torch.float64)
    out = R.sigmoid_cross_entropy_with_logits(lg, torch.full_like(lg, t))
    ref = torch.tensor([max(v, 0) - v * t + math.log1p(math.exp(-abs(v))) for v in x], dtype=torch.float64)
    assert torch.isfinite(out).all()
    assert torch.allclose(out, ref, atol=1e-12)
