"""MI355X-native Image Analogies best-match core (drop-in for flair2005/image-analogies-python).

The reference's modules keep their names and signatures here:
    config          parameters (reference config.py)
    img_preprocess  YIQ / remap / pyramids / B' init / index codec (reference img_preprocess.py)
    algorithms      feature layout, FLANN-compatible exact index, matching API (reference algorithms.py)
    image_analogies img_setup / image_analogies_main (reference image_analogies.py)
and run the hot path (per-level best-match synthesis) as hand-written gfx950 HIP kernels in
libia.so through a ctypes C ABI (include/ia.h).  Import as `ia_amd` (see ia_amd.py at the repo
root, which maps this hyphenated directory to that package name).
"""
__version__ = '0.1.0'
