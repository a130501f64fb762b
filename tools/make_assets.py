"""Decode the reference's texture asset and unit-test images into committed data.

The reference decodes earthmap.jpg with Go's image/jpeg at run time
(imageLoader.go:29-46).  Go is not available here, so the texture is decoded
once with PIL and committed as a binary PPM (P6) that the host scene code reads
(host_scenes.cpp load_image_texture).  earthmap.jpg is 4:4:4 sampled; PIL and
Go agree on the 5x5 PNG fixture exactly and on JPEGs within a few LSB
(SURVEY.md §4), so texel parity with the Go decoder is +-3/255, not exact.

Usage: python tools/make_assets.py [/root/reference]
"""
import json
import os
import sys

from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def to_ppm(src, dst):
    im = Image.open(src).convert("RGB")
    w, h = im.size
    with open(dst, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(im.tobytes())
    return w, h


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    os.makedirs(os.path.join(REPO, "assets"), exist_ok=True)
    w, h = to_ppm(os.path.join(ref, "earthmap.jpg"), os.path.join(REPO, "assets", "earthmap.ppm"))
    print("earthmap.ppm", w, h)
    # PIL decodes of the reference's 5x5 loader fixtures (imageLoader_test.go:9-30)
    out = {}
    for name in ("test.png", "test.jpg"):
        im = Image.open(os.path.join(ref, "internal", "imageloader", name)).convert("RGB")
        out[name] = {"w": im.size[0], "h": im.size[1], "rgb": list(im.tobytes())}
    with open(os.path.join(REPO, "tests", "golden", "imageloader_pil_decode.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
