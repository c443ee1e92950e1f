"""Loss-parity bound of the training-step tests, pinned by an fp64 run of the oracle.

The north-star bound is 1e-3 relative to the reference.  The reference's own fp32 arithmetic is measured
against an fp64 run of the same oracle step: where the fp32 reference itself drifts from fp64 by more
than that (the consistency loss after an optimizer step is (student - EMA teacher)^2 with the two models
1 % apart, and back-propagation through ~60 BatchNorm layers amplifies fp32 rounding in the gradients
that moved the student), the HIP result must stay within 2x the reference's own drift.  Step 0 (forward
arithmetic only, no optimizer step yet) always gets the plain 1e-3 bound.
"""


def loss_bound(r32, r64, strict=False, rel=1e-3, atol=1e-7):
    drift = abs(r32 - r64)
    return (rel * abs(r64) if strict else max(rel * abs(r64), 2.0 * drift)) + atol


def check_losses(hip, r32, r64, names=('sup', 'unsup')):
    """hip, r32, r64: per-step tuples of losses.  Returns the report lines; raises on a violation."""
    lines, bad = [], []
    for k, (h, a, b) in enumerate(zip(hip, r32, r64)):
        for n, hv, av, bv in zip(names, h, a, b):
            lim = loss_bound(av, bv, strict=(k == 0))
            err = abs(hv - bv)
            lines.append(f'step {k} {n}: hip {hv:.9g} ref32 {av:.9g} ref64 {bv:.9g} | |hip-64| {err:.3e} '
                         f'|ref32-64| {abs(av - bv):.3e} bound {lim:.3e} (rel {err / (abs(bv) + 1e-30):.2e})')
            if not err <= lim:
                bad.append(lines[-1])
    print('\n'.join(lines))
    assert not bad, bad
    return lines


def tensor_outliers(got, ref32, ref64, refp=None, rel=1e-3, floor=None, factor=2.0):
    """Per-tensor parity of parameters / gradients after a few optimizer steps: max |got - ref64| relative to
    the tensor's scale must stay within max(rel, 2x the fp32 oracle's drift, 2x the drift of an fp64 run on
    inputs perturbed by ~1e-6 (ReLU / max-pool switches of tiny-batch activations)).  Dicts of numpy
    arrays; `floor` (a global scale) keeps mathematically-zero tensors (a bias feeding a BatchNorm) from
    being judged on rounding noise; `factor` (default 2) multiplies the two drifts.  Returns the violating
    (name, err, drift32, drift_pert) rows."""
    import numpy as np
    bad = []
    for k, b in ref64.items():
        b = np.asarray(b, np.float64)
        if not np.issubdtype(b.dtype, np.floating):
            continue
        scale = max(float(np.abs(b).max()), floor or 0.0) + 1e-12
        e = float(np.abs(np.asarray(got[k], np.float64) - b).max()) / scale
        d32 = float(np.abs(np.asarray(ref32[k], np.float64) - b).max()) / scale
        dp = float(np.abs(np.asarray(refp[k], np.float64) - b).max()) / scale if refp is not None else 0.0
        if e > max(rel, factor * d32, factor * dp):
            bad.append((k, e, d32, dp))
    return bad
