"""Host image decode for the Node shim (js/babylon_pt.js): PNG / JPEG bytes on stdin -> 8-byte
header (width, height: uint32 little-endian) + RGBA8 rows top first on stdout.

The glTF loader hands the shim the map files' bytes (Texture.updateURL); Node has no JPEG decoder,
so the shim uses the Python host's (python/pt_assets.py decode_rgba8: Pillow, libjpeg-turbo with
its default IDCT and fancy upsampling - a browser's decoder is not pinned)."""
import io
import struct
import sys

import numpy as np
from PIL import Image


def main():
    data = sys.stdin.buffer.read()
    im = np.asarray(Image.open(io.BytesIO(data)).convert("RGBA"), dtype=np.uint8)
    sys.stdout.buffer.write(struct.pack("<II", im.shape[1], im.shape[0]))
    sys.stdout.buffer.write(np.ascontiguousarray(im).tobytes())


if __name__ == "__main__":
    main()
