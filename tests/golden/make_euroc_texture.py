"""Builds tests/golden/euroc_texture.npz — the plane texture of the C2-sized photometric problems (BASELINE.json
configs[1]: "EuRoC V1_01_easy photometric BA, 50 keyframes").  Four cam0 frames of the reference's own EuRoC V1
subset (/root/reference/data/euroc_V1/<timestamp>_0.jpg, 752×480 u8 gray), decoded with PIL here, tiled 2×2 into one
1504×960 u8 image (data, not code; the GPU box never reads the reference).  synth.make_problem(texture="euroc")
ray-casts every keyframe onto a plane carrying this texture, so the rendered frames are real EuRoC image content and
the photometric residual at the true state is ~0.

    python tests/golden/make_euroc_texture.py [/root/reference/data/euroc_V1]
"""
import os
import sys

import numpy as np
from PIL import Image

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/euroc_V1"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "euroc_texture.npz")


def main():
    names = sorted(n for n in os.listdir(SRC) if n.endswith("_0.jpg"))
    pick = [names[int(i)] for i in np.linspace(0, len(names) - 1, 4)]
    tiles = [np.asarray(Image.open(os.path.join(SRC, n)).convert("L"), np.uint8) for n in pick]
    assert all(t.shape == (480, 752) for t in tiles), [t.shape for t in tiles]
    mosaic = np.block([[tiles[0], tiles[1]], [tiles[2], tiles[3]]])
    np.savez_compressed(OUT, texture=mosaic, frames=np.array(pick))
    print(OUT, mosaic.shape, pick)


if __name__ == "__main__":
    main()
