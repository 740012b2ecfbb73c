"""Generate tests/golden/fractal_ref.npz from the reference's own Mandelbrot render.

Input (read here, in the build container only; never at test time):
  /root/reference/Notes/README/fractal.png -- the 1024x1024 RGBA8 image written by
  src/examples/image_with_compute_shader.rs:150 (`save_image(..., "target/fractal.png")`)
  after dispatching its inline shader (:19-47) over a R8G8B8A8_UNORM storage image (:65-70).
  That shader is assets/shaders/mandelbrot.comp:12-33 at the default camera
  (position [0, 0], scale 1: src/mandelbrot/config.rs:11-12), where `c / 1.0 + 0.0` is exact,
  so the two compute the same c for every pixel.

Output: the grey channel (R; G and B are equal and alpha is 255 on every pixel, checked
here) as a 1024x1024 uint8 array ``grey``.  The data are the reference's output values, not
its source.
"""
import os
import sys

import numpy as np
from PIL import Image

SRC = "/root/reference/Notes/README/fractal.png"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fractal_ref.npz")


def main():
    img = np.asarray(Image.open(SRC).convert("RGBA"))
    assert img.shape == (1024, 1024, 4), img.shape
    assert (img[..., 0] == img[..., 1]).all() and (img[..., 0] == img[..., 2]).all()
    assert (img[..., 3] == 255).all()
    np.savez_compressed(OUT, grey=img[..., 0].copy(), width=1024, height=1024,
                        position=np.array([0.0, 0.0], np.float32), scale=np.float32(1.0))
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    sys.exit(main())
