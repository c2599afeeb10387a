"""Parity rules between a GMRES run and the oracle / golden record.

Stated tolerances (the north-star's "within a stated fp tolerance"). be(c)
is the per-restart backward error r/(||b|| + ||A||_F ||x||) of cycle c
(IterUtil.hpp:37-61), s(k+1) the per-step Arnoldi residual.

fp64 Arnoldi with an fp64 preconditioner (mode baseline):
  * same final status, same restart index i and total iteration count;
  * per-step |s(k+1)|, cycle 0:  |Δ| <= 1e-8 |s_ref| + 1e-12 ||M^-1 b||;
    later cycles:               |Δ| <= 1e-5 |s_ref| + 1e-10 ||M^-1 b||;
  * every cycle's backward error: |Δ| <= 1e-5 be_ref + 1e-15;
  * x, first 16 entries: |Δ| <= 1e-12 max|x_ref| + 0.25 e_ref,
    sum: |Δ| <= 1e-12 max(|Σx_ref|, max|x_ref|) + 1.0 sqrt(n) e_ref,
    where e_ref = errNorm = ||x_ref - x_true||_2 of the reference run only:
    each entry of the GPU's x must lie within a quarter of the reference's
    own error of the reference's x (a bound that does not grow with the run
    under test;
    |Δ| <= e_ref + e_got holds for any two runs, so a bound with e_got in it
    can never fail). Rounding-level differences (an ill-conditioned C1
    differs at 2e-12 relative) sit far inside it;
  * final resNorm within a factor 1.2 and errNorm within a factor 2, both
    above a floor: 64 eps (||b|| + ||A||_F ||x||) for resNorm, 64 eps
    sqrt(n) max|x| for errNorm (a 2-norm of n eps-level entry errors).
fp32 Arnoldi, or fp64 Arnoldi whose vectors pass through an fp32
preconditioner every step (modes mixed, single, mixed-half, single-prec):
  * same final status; restart index within ±1;
  * cycle-0 history |Δ| <= 1e-3 |s_ref| + 1e-5 ||M^-1 b||;
  * every cycle both runs reached (all but the last when the restart
    counts differ): max(be, F) within a factor 3 of max(be_ref, F), with
    the floor F = 1e-14 (fp64 residual) or 1e-6 (mode single, fp32
    residual) — the restarts of an fp32 cycle contract the error by
    amounts that differ with the fp32 rounding, never by more than that;
  * x: the rule above with 1e-9 (fp64 outer) / 1e-5 (single) relative,
    0.5 e_ref for the head and 2.5 sqrt(n) e_ref for the sum (same restart
    count only): the fp32 cycle's corrections differ in rounding, so the
    iterates agree only to a fraction of the error they carry;
  * final resNorm within a factor 10 (above the floor); errNorm at most
    10x the reference's (a more accurate x than the oracle's is not a
    parity failure: forward error at convergence depends on conditioning);
  * when converged, the final backward error is <= tol.
Live-oracle comparisons of fp32 Arnoldi on large inputs (compare_mkl, round
5) compare with the MKL oracle two-sidedly. Round 6 adds the GPU's fp32
accumulation class (accum="f32": every partial sum of the fp32 Arnoldi in
fp32, the reference's cblas_s* / mkl_sparse_s_mv class) and, for it, an
envelope without the fp64-summing loop kernels: MKL at MKL_THREADS and the
oracle's "pair32" loop mode (the same fp32-accumulating operations, long
reductions in pairwise order). Within the fp32 class the accumulation ORDER
sets how fast plain CGS loses orthogonality (BAND-300k m = 100, cycle-1
backward error: one sequential fp32 chain 1.5e-7, MKL 6.0e-9, pairwise fp32
4.5e-10, GPU f32 3.9e-10, fp64 sums 2.4e-10; stencil27p: 1.4e-7, 2.7e-8,
8.07e-9, GPU f32 8.07e-9, 8.06e-9 -- profiles/r06_accum/), and a GPU
reduction is a tree, as is the reference's own GPU backend's (cublasSdot /
Sgemv, kernels_cuda.cpp:132,160). The oracle's MKL is pinned to one
code branch (MKL_CBWR=COMPATIBLE, set by oracle/binding.py: conditional
numerical reproducibility) and run at fixed thread counts (MKL_THREADS), so
its bits no longer depend on the host: the same digests on the build
container's Xeon and the GPU box's EPYC at 1, 4 and 8 threads
(profiles/r05_oracle_cnr/; round 4 had seen its cycle-1 backward error move
3-12x between the two, profiles/r04_oracle_backends.txt). What CNR does not
remove is the accuracy class: MKL's fp32 sgemv sums in fp32, so with plain
CGS (one orthogonalisation pass) a large fp32 solve loses orthogonality
faster than the HIP kernels, which sum in fp64 -- BAND-300k at m = 100:
cycle-1 backward error 6.0e-9 (MKL, any thread count) vs 2.4e-10 (GPU);
with CGSR the two agree to 10 %. So each cycle's backward error must lie in
the envelope of the kernels_mkl.cpp arithmetic evaluated by the oracle --
MKL at each of MKL_THREADS and the oracle's loop kernels (the same
operations with fp32 products summed in fp64 in index order) -- widened by
the factor 3 of the rule above ([min/3, 3 max]); everything else follows
compare() against the 1-thread MKL run (the reference's serial
arithmetic).
Measured margins behind these numbers: tools/parity_margins.py over the
168 golden records on the fused and operator-surface engines
(profiles/r02_parity_margins.txt; the x terms against e_ref alone:
profiles/r03_parity_margins.txt, head <= 0.038 / 0.16 e_ref and sum <=
0.41 / 1.24 sqrt(n) e_ref for fp64 / fp32 Arnoldi).
"""
import numpy as np


def _arr(x):
    return np.asarray(x, dtype=np.float64)


def _ratio_ok(a, b, factor):
    a, b = float(a), float(b)
    if a == b:
        return True
    if not (np.isfinite(a) and np.isfinite(b)) or a <= 0 or b <= 0:
        return False
    return max(a / b, b / a) <= factor


def compare(ref: dict, got, mode: str, tol: float, rlen: int, label: str = "", envelope=None):
    """envelope: None, or a list of oracle Results of the same solve (MKL at
    MKL_THREADS) whose per-cycle backward errors bound got's (fp32 Arnoldi
    rule, see the module docstring) and whose restart counts widen the +-1
    rule; ref stays the reference for every other check."""
    fp64 = mode == "baseline"
    assert got.status == ref["status"], f"{label}: status {got.status} vs {ref['status']}"
    minvb = float(ref["minvb_norm"])
    s_ref, s_got = _arr(ref["step_res"]), _arr(got.step_res)
    cyc = np.asarray(got.step_cycle)
    be_ref = _arr(ref["cyc_r_norm"]) / _arr(ref["cyc_normalization"])
    be_got = _arr(got.cyc_r_norm) / _arr(got.cyc_normalization)
    x_head_ref = _arr(ref["x_head"]) if "x_head" in ref else None
    xscale = float(np.max(np.abs(x_head_ref))) if x_head_ref is not None and len(x_head_ref) else 0.0
    if fp64:
        assert got.restarts == ref["restarts"], f"{label}: restarts {got.restarts} vs {ref['restarts']}"
        assert got.total_iters == ref["total_iters"], f"{label}: iters {got.total_iters} vs {ref['total_iters']}"
        assert len(s_got) == len(s_ref)
        c0 = cyc == 0
        d = np.abs(s_got - s_ref)
        assert np.all(d[c0] <= 1e-8 * s_ref[c0] + 1e-12 * minvb), f"{label}: cycle-0 history {d[c0].max():.3e}"
        assert np.all(d[~c0] <= 1e-5 * s_ref[~c0] + 1e-10 * minvb), f"{label}: history {d[~c0].max():.3e}"
        assert np.all(np.abs(be_got - be_ref) <= 1e-5 * be_ref + 1e-15), f"{label}: backward errors"
        x_rtol, e_w, e_ws, norm_factor = 1e-12, 0.25, 1.0, (1.2, 2.0)
    else:
        restarts = [ref["restarts"]] + ([int(r.restarts) for r in envelope] if envelope else [])
        assert min(abs(got.restarts - r) for r in restarts) <= 1, f"{label}: restarts {got.restarts} vs {restarts}"
        k = min(rlen, len(s_ref), len(s_got))
        d = np.abs(s_got[:k] - s_ref[:k])
        assert np.all(d <= 1e-3 * s_ref[:k] + 1e-5 * minvb), f"{label}: cycle-0 history {d.max():.3e}"
        floor = 1e-6 if mode == "single" else 1e-14
        if envelope:
            ok, msg = mkl_envelope_ok(envelope, got, mode)
            assert ok, f"{label}: {msg}"
        else:
            nc = min(len(be_ref), len(be_got)) - (0 if got.restarts == ref["restarts"] else 1)
            for c in range(max(nc, 0)):
                assert _ratio_ok(max(be_got[c], floor), max(be_ref[c], floor), 3.0), \
                    f"{label}: cycle {c} backward error {be_got[c]:.3e} vs {be_ref[c]:.3e}"
        if got.status == "converged":
            assert be_got[-1] <= tol, f"{label}: final backward error {be_got[-1]:.3e} > {tol}"
        x_rtol, e_w, e_ws = (1e-5 if mode == "single" else 1e-9), 0.5, 2.5
        norm_factor = (10.0, 10.0)
    same_cycles = got.restarts == ref["restarts"]
    e_ref, e_got = float(ref.get("err_norm") or 0.0), float(getattr(got, "err_norm", 0.0) or 0.0)
    if x_head_ref is not None and same_cycles and xscale > 0:
        dx = np.max(np.abs(_arr(got.x[:len(x_head_ref)]) - x_head_ref))
        bound = x_rtol * xscale + e_w * e_ref
        assert dx <= bound, f"{label}: x head differs by {dx:.3e} (bound {bound:.3e}, scale {xscale:.3e})"
        xs_ref = float(ref["x_sum"])
        ds = abs(float(np.sum(got.x)) - xs_ref)
        bound = x_rtol * max(abs(xs_ref), xscale) + e_ws * np.sqrt(len(got.x)) * e_ref
        assert ds <= bound, f"{label}: x sum differs by {ds:.3e} (bound {bound:.3e})"
    if "res_norm" in ref and same_cycles and hasattr(got, "res_norm"):
        norm_last = float(_arr(ref["cyc_normalization"])[-1])
        rf = 64 * np.finfo(np.float64).eps * norm_last
        assert _ratio_ok(max(got.res_norm, rf), max(ref["res_norm"], rf), norm_factor[0]), \
            f"{label}: resNorm {got.res_norm:.3e} vs {ref['res_norm']:.3e}"
        if e_ref:
            # errNorm is a 2-norm over n entries, each carrying eps-level
            # rounding: its floor grows with sqrt(n)
            ef = 64 * np.finfo(np.float64).eps * np.sqrt(len(got.x)) * xscale
            if fp64:
                assert _ratio_ok(max(e_got, ef), max(e_ref, ef), norm_factor[1]), \
                    f"{label}: errNorm {e_got:.3e} vs {e_ref:.3e}"
            else:
                assert e_got <= norm_factor[1] * max(e_ref, ef), f"{label}: errNorm {e_got:.3e} vs {e_ref:.3e}"


# the oracle's MKL thread counts of compare_mkl (fixed, so the envelope is
# the same on every host: the MKL branch is pinned by MKL_CBWR)
MKL_THREADS = (1, 4, 8)


def mkl_envelope_ok(refs, got, mode: str, factor: float = 3.0):
    """(ok, message): every cycle's backward error of got (above the floor)
    within [min_T be_T / factor, factor max_T be_T] over the runs refs, for
    the cycles every run reached (all but the last when restart counts
    differ)."""
    floor = 1e-6 if mode == "single" else 1e-14
    be_got = _arr(got.cyc_r_norm) / _arr(got.cyc_normalization)
    bes = [_arr(r.cyc_r_norm) / _arr(r.cyc_normalization) for r in refs]
    same = all(r.restarts == got.restarts for r in refs)
    nc = min([len(be_got)] + [len(b) for b in bes]) - (0 if same else 1)
    for c in range(max(nc, 0)):
        lo = min(max(b[c], floor) for b in bes)
        hi = max(max(b[c], floor) for b in bes)
        g = max(be_got[c], floor)
        if not (np.isfinite(g) and lo / factor <= g <= factor * hi):
            return False, f"cycle {c} backward error {be_got[c]:.3e} outside [{lo / factor:.3e}, {factor * hi:.3e}]"
    return True, ""


def compare_mkl(oracle, mpg, A, b, xt, got, opts: dict, label: str = "", runs: dict = None,
                extra: tuple = ("loops",)):
    """Two-sided parity with the MKL oracle (module docstring): the oracle at
    each of MKL_THREADS (pinned MKL branch) and on the loop-kernel modes in
    `extra`; got compared with the 1-thread MKL run, its per-cycle backward
    errors inside the runs' envelope. The fp64-accumulating GPU class takes
    extra=("loops",) (fp32 products summed in fp64: its own class); a GPU run
    in the reference's fp32 class (accum="f32") takes
    extra=("pair32",): the same fp32-accumulating arithmetic in a tree order,
    the order of a GPU reduction (oracle/binding.py LOOP_MODES). runs: a
    cache {threads or loop mode: Result}."""
    runs = {} if runs is None else runs
    opts = {k: v for k, v in opts.items() if k != "accum"}  # (the oracle's class is its backend's)
    for t in MKL_THREADS:
        if t not in runs:
            runs[t] = oracle.solve(mpg, A, b, xt, backend="mkl", threads=t, **opts)
    refs = [runs[t] for t in MKL_THREADS]
    for mode in extra:
        if mode not in runs:
            runs[mode] = oracle.solve(mpg, A, b, xt, backend=mode, threads=1, **opts)
        refs.append(runs[mode])
    compare(as_ref(refs[0]), got, opts["mode"], opts["tol"], opts["rlen"], label, envelope=refs)
    return runs


def golden_envelope(oracle, mpg, A, b, xt, rec: dict, opts: dict):
    """The envelope of a golden record (made by the oracle's pinned MKL
    branch, 1 thread): the record and the oracle's loop kernels run live on
    the same inputs -- the fp64-accumulating summation class of the HIP
    kernels. Near convergence an fp32 Arnoldi's attainable accuracy moves
    with the summation order: convdiff32 at m = 100 ends cycle 2 at 5.5e-14
    under MKL and 6.2e-15 on the loops (GPU: 6.6e-15)."""
    from types import SimpleNamespace

    g = SimpleNamespace(cyc_r_norm=rec["cyc_r_norm"], cyc_normalization=rec["cyc_normalization"],
                        restarts=rec["restarts"])
    return [g, oracle.solve(mpg, A, b, xt, backend="loops", threads=1, **opts)]


def not_worse_than(ref, got, mode: str, label: str = "", factor: float = 3.0):
    """One-sided bound: every cycle's backward error of `got` at most
    `factor` x the reference run's (above the compare() floor); a GPU run
    more accurate than an fp32-summing oracle passes."""
    floor = 1e-6 if mode == "single" else 1e-14
    be_ref = _arr(ref.cyc_r_norm) / _arr(ref.cyc_normalization)
    be_got = _arr(got.cyc_r_norm) / _arr(got.cyc_normalization)
    nc = min(len(be_ref), len(be_got)) - (0 if got.restarts == ref.restarts else 1)
    for c in range(max(nc, 0)):
        assert be_got[c] <= factor * max(be_ref[c], floor), \
            f"{label}: cycle {c} backward error {be_got[c]:.3e} > {factor} x {be_ref[c]:.3e}"


def as_ref(result) -> dict:
    """Turn a live oracle Result into the golden-record shape."""
    return dict(status=result.status, restarts=result.restarts, total_iters=result.total_iters,
                minvb_norm=result.minvb_norm, step_res=result.step_res, step_cycle=result.step_cycle,
                cyc_r_norm=result.cyc_r_norm, cyc_normalization=result.cyc_normalization,
                res_norm=result.res_norm, err_norm=result.err_norm,
                x_head=np.asarray(result.x[:16]), x_sum=float(np.sum(result.x)))
