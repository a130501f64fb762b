"""Parity metrics between the HIP path and the CPU oracle (shared by tests)."""
import numpy as np


def compare(gpu_img, ref_img):
    """Per-pixel agreement statistics on linear RGB and on the 8-bit output."""
    import go_raytracer_amd as rt
    g = np.asarray(gpu_img, np.float64)
    r = np.asarray(ref_img, np.float64)
    fin = np.isfinite(g) & np.isfinite(r)
    diff = np.where(fin, np.abs(g - r), np.where(np.isnan(g) == np.isnan(r), 0.0, np.inf))
    tol = 1e-3 * np.maximum(1.0, np.nan_to_num(np.abs(r), nan=1.0, posinf=1.0))
    q_g = rt.quantize(gpu_img).astype(np.int32)
    q_r = rt.quantize(ref_img).astype(np.int32)
    dq = np.abs(q_g - q_r)
    return {
        "frac_close": float(np.mean(diff <= tol)),
        "max_abs": float(np.max(np.where(np.isfinite(diff), diff, 0))),
        "mean_abs": float(np.mean(np.where(np.isfinite(diff), diff, 0))),
        "q_equal": float(np.mean(dq == 0)),
        "q_within2": float(np.mean(dq <= 2)),
        "mean_gpu": g[np.isfinite(g)].mean() if np.isfinite(g).any() else float("nan"),
        "mean_ref": r[np.isfinite(r)].mean() if np.isfinite(r).any() else float("nan"),
    }
