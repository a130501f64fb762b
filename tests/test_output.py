"""Output quantisation: PrintColor (vec/color.go:23-46) and the PPM P3 stream."""
import numpy as np


def test_quantize_matches_oracle_print_color(rt, oracle):
    rng = np.random.default_rng(1)
    vals = np.concatenate([rng.uniform(-0.5, 2.0, 3000), [0.0, -0.0, 0.25, 1.0, 0.99999 ** 2,
                                                          np.nan, np.inf, -np.inf, 1e30, 1e-30]])
    vals = vals[: len(vals) // 3 * 3].astype(np.float32).reshape(-1, 3)
    q = rt.quantize(vals)
    for row, qr in zip(vals, q):
        assert oracle.print_color(*map(float, row)) == "%d %d %d\n" % tuple(qr)


def test_quantize_known_answers(rt):
    q = rt.quantize(np.array([[0.25, np.nan, np.inf]], np.float32))
    assert q.tolist() == [[128, 0, 255]]  # sqrt(.25)*256; NaN -> 0; Inf clamps to .99999


def test_ppm_format(rt):
    img = np.zeros((2, 3, 3), np.float32)
    img[0, 0] = [1, 1, 1]
    txt = rt.format_ppm(img).decode()
    lines = txt.split("\n")
    assert lines[0] == "P3" and lines[1] == "3 2" and lines[2] == "255"  # camera.go:160
    assert lines[3] == "255 255 255" and lines[4] == "0 0 0"
    assert txt.endswith("\n") and len(lines) == 3 + 6 + 1
