"""Parity metrics between the HIP path and the CPU oracle (shared by tests).

Set PARITY_LOG=path to append every comparison (test id + metrics) as a JSON line:
that is how the thresholds in the tests were calibrated (DESIGN.md "Parity")."""
import json
import os

import numpy as np


def compare(gpu_img, ref_img, label=None):
    """Per-pixel agreement statistics on linear RGB and on the 8-bit output.
    `label` tags the PARITY_LOG line (e.g. "fp32_oracle" for the oracle's fp32 twin
    against its fp64 path: what an fp32 evaluation of the reference itself reaches)."""
    import go_raytracer_amd as rt
    g = np.asarray(gpu_img, np.float64)
    r = np.asarray(ref_img, np.float64)
    fin = np.isfinite(g) & np.isfinite(r)
    # non-finite pairs agree only when identical (both NaN, or the same infinity)
    same = (np.isnan(g) & np.isnan(r)) | (g == r)
    diff = np.where(fin, np.abs(g - r), np.where(same, 0.0, np.inf))
    # |delta| <= 2^-10 * max(1, |ref|)
    tol = 2.0 ** -10 * np.maximum(1.0, np.nan_to_num(np.abs(r), nan=1.0, posinf=1.0))
    q_g = rt.quantize(gpu_img).astype(np.int32)
    q_r = rt.quantize(ref_img).astype(np.int32)
    dq = np.abs(q_g - q_r)
    m = {
        "frac_close": float(np.mean(diff <= tol)),
        "max_abs": float(np.max(np.where(np.isfinite(diff), diff, 0))),
        "mean_abs": float(np.mean(np.where(np.isfinite(diff), diff, 0))),
        "q_equal": float(np.mean(dq == 0)),
        "q_within2": float(np.mean(dq <= 2)),
        "mean_gpu": g[np.isfinite(g)].mean() if np.isfinite(g).any() else float("nan"),
        "mean_ref": r[np.isfinite(r)].mean() if np.isfinite(r).any() else float("nan"),
    }
    if os.environ.get("PARITY_LOG"):
        with open(os.environ["PARITY_LOG"], "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", ""),
                                **({"label": label} if label else {}),
                                **{k: float(v) for k, v in m.items()}}) + "\n")
    return m


P1_BAR = 0.995

# >= 99.5 % of linear-RGB channels within 2^-10 * max(1, |ref|)
# ("frac_close") and of 8-bit outputs equal ("q_equal").  Every scene is held to it
# except the one named here, with its measured GPU result (round 6,
# profiles/r6_parity_final.jsonl): its paths are chaotic, and fp32 and fp64 paths fork after
# a few bounces whatever the implementation (tools/fork_census.py: 168 of 196 forked samples
# part at the 4th vertex or later, none at the camera ray).
# (Round 6: the `cluster` feature scene, 200 small spheres, renders at 64 x 64 x 32 and meets
# P1 itself, q_equal 0.9990 against 0.995 on 12,288 channels, ~14 sigma; at 32 x 32 x 16 it
# had needed its own 0.990 bar.)
P1_EXCEPTIONS = {
    # C5, the 1M-triangle metal knot at 1920x1080x1024 (row subsample, 17 rows each):
    # frac_close 0.99315 / 0.99314, q_equal 0.99146 / 0.99175 on the two row sets (round 5:
    # 0.9933 / 0.9931 and 0.9914 / 0.9916).  The GPU render and the oracle are deterministic,
    # so the margin does not vary from box to box; it moves only with the arithmetic.
    "model": {"frac_close": 0.993, "q_equal": 0.990},
}


def p1_bar(name, key):
    """The parity bar for metric `key` of scene `name`: P1's 0.995, or the named
    exception's bar above."""
    return P1_EXCEPTIONS.get(name, {}).get(key, P1_BAR)
