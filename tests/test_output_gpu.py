"""On-device output path: rt_quantize_device and
rt_format_ppm_device must produce exactly the bytes of the host PrintColor /
P3 writer (vec/color.go:23-46, camera.go:160), which test_output.py pins to the
oracle's PrintColor."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def edge_values():
    q = np.arange(0, 257, dtype=np.float64)
    sq = (q * q / 65536.0).astype(np.float32)  # exact squares: sqrt lands on q/256
    up = np.nextafter(sq, np.float32(np.inf))
    dn = np.nextafter(sq, np.float32(-np.inf))
    special = np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 1e-45, -1e-45, 1e-38, 0.99999 ** 2,
                        np.nextafter(np.float32(0.99999 ** 2), np.float32(1)), 1.0, 3e38],
                       np.float32)
    rnd = np.random.default_rng(7).uniform(-0.5, 2.0, 30000).astype(np.float32)
    v = np.concatenate([sq, up, dn, special, rnd]).astype(np.float32)
    return v[: len(v) // 3 * 3].reshape(-1, 3)


def test_quantize_device_bitwise(rt, gpu):
    import torch
    v = edge_values()
    got = rt.quantize_device(torch.from_numpy(v).cuda()).cpu().numpy()
    assert np.array_equal(got, rt.quantize(v))


@pytest.mark.parametrize("hw", [(1, 1), (2, 3), (1, 1000), (7, 333), (800, 800), (1080, 1920)])
def test_format_ppm_device_bitwise(rt, gpu, hw):
    import torch
    h, w = hw
    rng = np.random.default_rng(h * 7919 + w)
    img = rng.uniform(-0.1, 1.3, (h, w, 3)).astype(np.float32)
    img.reshape(-1)[:: 97] = np.nan
    assert rt.format_ppm_device(torch.from_numpy(img).cuda()) == rt.format_ppm(img)


@pytest.mark.parametrize("misalign", [1, 2, 3])
def test_format_ppm_device_unaligned_output(rt, gpu, misalign):
    import torch
    img = np.random.default_rng(misalign).uniform(0, 1, (37, 41, 3)).astype(np.float32)
    d = torch.from_numpy(img).cuda()
    n = int(rt.lib().rt_format_ppm_device(d.data_ptr(), 41, 37, None, 0, 0, None))
    buf = torch.full((n + 8,), 0xAB, dtype=torch.uint8, device="cuda")
    got = rt.lib().rt_format_ppm_device(d.data_ptr(), 41, 37, C.c_void_p(buf.data_ptr() + misalign),
                                        n, 0, None)
    assert got == n
    b = buf.cpu().numpy().tobytes()
    assert b[misalign:misalign + n] == rt.format_ppm(img)
    assert set(b[:misalign]) == {0xAB} and set(b[misalign + n:]) == {0xAB}  # nothing outside


def test_too_small_buffer_is_an_error_not_an_overrun(rt, gpu):
    import torch
    img = torch.rand(16, 16, 3, device="cuda")
    n = int(rt.lib().rt_format_ppm_device(img.data_ptr(), 16, 16, None, 0, 0, None))
    buf = torch.full((n,), 0xAB, dtype=torch.uint8, device="cuda")
    rc = rt.lib().rt_format_ppm_device(img.data_ptr(), 16, 16, C.c_void_p(buf.data_ptr()), n - 10,
                                       0, None)
    assert rc == -1
    assert set(buf.cpu().numpy()[n - 10:].tolist()) == {0xAB}


def test_render_to_ppm_on_device(rt, gpu):
    """Render into a device tensor and format it there: same bytes as the host path."""
    import torch
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = 64, 16
    W, H, _ = cam.image_size()
    out = torch.empty(H, W, 3, dtype=torch.float32, device="cuda")
    with rt.Scene(t, w, l) as sc:
        sc.render_device(cam, out.data_ptr(), seed=5,
                         stream=torch.cuda.current_stream().cuda_stream)
        img, _ = sc.render(cam, seed=5)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), img)
    assert rt.format_ppm_device(out) == rt.format_ppm(img)


def test_progress_while_rendering(rt, gpu):
    """rt_progress polled from another thread sees the render advance slice by slice
    (the reference's progress bar, camera.go:106-108); slicing leaves the image
    bit-identical and progress reports completion afterwards."""
    import threading
    import time
    t, cam, w, l = rt.demo_scene("cornell")
    cam.Width, cam.SamplesPerPixel = 800, 1024
    seen = []
    with rt.Scene(t, w, l) as sc:
        ref, _ = sc.render(cam, seed=1)
        assert sc.progress() == (655360000, 655360000)
        stop = threading.Event()

        def poll():
            while not stop.is_set():
                seen.append(sc.progress())
                time.sleep(0.0005)
        th = threading.Thread(target=poll)
        th.start()
        img, st = sc.render(cam, seed=1, progress_slices=16)
        stop.set()
        th.join()
        done, total = sc.progress()
    assert np.array_equal(img, ref, equal_nan=True)
    assert total == st["samples"] == done
    mid = sorted({d for d, tt in seen if 0 < d < total})
    assert len(mid) >= 4, seen[:40]
    assert all(0 <= d <= tt for d, tt in seen)
