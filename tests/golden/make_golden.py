#!/usr/bin/env python3
"""Regenerates the golden framebuffers of tests/golden with the CPU oracle
(oracle/bih_oracle.c, the strict-IEEE restatement of the reference's render
path; SURVEY 8c: the reference itself cannot run here, so these are the
oracle's outputs, checked bit-exactly against the HIP path on the GPU box).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))

CASES = [("cornell_256x256_f0.npy", "cornell", 256, 256, 0),
         ("cornell_256x256_f7.npy", "cornell", 256, 256, 7),
         ("dodeca_64x64_f0.npy", "dodeca", 64, 64, 0),
         ("bih1_dodeca_640x480_f0.npy", "bih1_dodeca", 640, 480, 0)]


def main():
    import oracle
    from conftest import edge_scenes
    scenes = edge_scenes()
    for fname, scene, w, h, frame in CASES:
        img, _ = oracle.OracleTree(scenes[scene]).render(w, h, spp=4, frame=frame, seed=1984)
        np.save(os.path.join(HERE, fname), img)
        print(fname, img.shape, len(np.unique(img)), "shades")


if __name__ == "__main__":
    main()
