"""Generate tests/golden/readme_blockmeans.npz from the reference's only rendered output.

Input (read here, in the build container only; never at test time):
  /root/reference/README/image-20240918152736292.png -- a 1022x1052 window capture of the
  reference rendering the Cornell box at 1024x1024, SPP=30 (README.md:14-15), with the
  games101 kernel.

Alignment (found by minimising the MSE of 5x5-box-blurred images against the oracle over
offsets in [-3, 3]^2; the minimum is unique): screenshot pixel (row r, col c) is image
pixel (y = r - 29, x = c + 1).  Rows 0-28 are the window title bar.  Image row 1023 and
columns 0 and 1023 are not visible.

Output: mean 8-bit RGB (scaled to [0, 1]) of the visible pixels of every 32x32 image block
(a 32x32x3 float32 array, ``blocks32``) and of every 16x16 block (``blocks16``), plus
the alignment constants; and (readme_pixels.npz) the aligned 8-bit frame itself, ``rgb``
(1024x1024x3 uint8, 0 where not visible) with its ``visible`` mask, for the per-pixel L2
statement (tests/test_oracle_reference.py).  The data are the reference's output values, not
its source.
"""
import os
import sys

import numpy as np
from PIL import Image

SRC = "/root/reference/README/image-20240918152736292.png"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "readme_blockmeans.npz")
OUT_PIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "readme_pixels.npz")
ROW0, COL_TO_X = 29, 1


def blocks(img, k):
    n = img.shape[0] // k
    return np.nanmean(img.reshape(n, k, n, k, 3).transpose(0, 2, 1, 3, 4).reshape(n, n, -1, 3),
                      axis=2)


def main():
    shot = np.asarray(Image.open(SRC).convert("RGB")).astype(np.float64) / 255.0
    assert shot.shape == (1052, 1022, 3), shot.shape
    img = np.full((1024, 1024, 3), np.nan)
    img[0:1052 - ROW0, COL_TO_X:COL_TO_X + 1022] = shot[ROW0:1052, 0:1022]
    np.savez_compressed(OUT, blocks32=blocks(img, 32).astype(np.float32),
                        blocks16=blocks(img, 16).astype(np.float32),
                        row0=ROW0, col_to_x=COL_TO_X, width=1024, height=1024, spp=30)
    print("wrote", OUT)
    raw = np.asarray(Image.open(SRC).convert("RGB"))
    rgb = np.zeros((1024, 1024, 3), np.uint8)
    vis = np.zeros((1024, 1024), bool)
    rgb[0:1052 - ROW0, COL_TO_X:COL_TO_X + 1022] = raw[ROW0:1052, 0:1022]
    vis[0:1052 - ROW0, COL_TO_X:COL_TO_X + 1022] = True
    np.savez_compressed(OUT_PIX, rgb=rgb, visible=vis, row0=ROW0, col_to_x=COL_TO_X)
    print("wrote", OUT_PIX, os.path.getsize(OUT_PIX), "bytes")


if __name__ == "__main__":
    sys.exit(main())
