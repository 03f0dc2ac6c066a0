"""Fixture generator -- TEST INFRASTRUCTURE ONLY.

Searches for the 36-triangle dodecahedron soup whose BIH is the reference's
own tree dump (reference BIH_Raytracer/BIH_Raytracer/BIH1.txt:1-348, copied to
tests/golden/reference_BIH1.txt) and writes the winner to
tests/golden/bih1_dodecahedron.npy (36 x 9 float32, fan order as searched).

Search space:
  * both axis-aligned dodecahedron orientations (every axis permutation or
    sign flip of a regular dodecahedron with cube-aligned vertices is one of
    the two; `variant` 0/1 of bihrt.scenes.dodecahedron);
  * every fan apex per face, 5^12 per orientation (every triangulation of a
    convex pentagon is a fan, so this covers every assimp
    aiProcess_Triangulate output, src/Model.cpp:13);
  * vertex precisions: f32 of the closed form; 6-significant-digit OBJ text
    (what Blender / most exporters write); closed form evaluated in f32.

The enumeration runs in bih1_search.c (gcc, OpenMP); every reported match is
re-checked here through the oracle library (oracle/bih_oracle.c ob_build).

Usage: python tests/golden/make_bih1_soup.py [--write]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))
sys.path.insert(0, ROOT)

from bihrt import scenes  # noqa: E402

DUMP = os.path.join(HERE, "reference_BIH1.txt")
OUT = os.path.join(HERE, "bih1_dodecahedron.npy")
META = os.path.join(HERE, "bih1_dodecahedron.json")


def vertex_sets(variant: int):
    """Yield (name, float32[20,3]) for each precision of one orientation."""
    _, faces, Vd = scenes.dodecahedron(variant=variant)   # float64 closed form
    yield "f32_of_f64", Vd.astype(np.float32), faces
    txt = np.array([[np.float32(float("%.6g" % x)) for x in row] for row in Vd], np.float32)
    yield "obj_6_significant", txt, faces
    # closed form evaluated in float32 arithmetic
    f = np.float32
    s = f(1) / np.sqrt(f(3))
    phi = (f(1) + np.sqrt(f(5))) / f(2)
    a32, b32, o32 = (f(1) / phi) * s, phi * s, s
    a64 = 1 / ((1 + 5 ** 0.5) / 2) / 3 ** 0.5
    b64 = ((1 + 5 ** 0.5) / 2) / 3 ** 0.5
    o64 = 1 / 3 ** 0.5

    def remap(x):
        ax = abs(x)
        for v64, v32 in ((a64, a32), (b64, b32), (o64, o32)):
            if abs(ax - v64) < 1e-9:
                return np.copysign(v32, x)
        return f(0)
    yield "closed_form_f32", np.array([[remap(x) for x in row] for row in Vd], np.float32), faces


def soup(V, faces, apex):
    tris = []
    for fc, st in zip(faces, apex):
        c = list(fc[st:]) + list(fc[:st])
        for k in range(1, 4):
            tris.append(np.concatenate([V[c[0]], V[c[k]], V[c[k + 1]]]))
    return np.ascontiguousarray(np.asarray(tris, np.float32))


def build_search() -> str:
    exe = os.path.join(tempfile.gettempdir(), "bih1_search")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-msse2",
                    "-mfpmath=sse", "-o", exe, os.path.join(HERE, "bih1_search.c"), "-lm"],
                   check=True)
    return exe


def dump_nodes():
    nodes = []
    for line in open(DUMP):
        line = line.strip()
        if line.startswith("NODE"):
            nodes.append({})
        elif ":" in line:
            k, v = [s.strip() for s in line.split(":", 1)]
            nodes[-1][k] = v
    return nodes


def tree_matches_dump(tris) -> int:
    """Number of the dump's 35 nodes the oracle's tree reproduces in all 8
    fields (clip planes compared at the dump's printed precision, %g)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    t = O.OracleTree(tris)
    if t.U != 36:
        return 0
    ok = 0
    for i, n in enumerate(dump_nodes()):
        fields = (int(n["parent"]) == int(t.parent[i]),
                  int(n["leftChild"]) == int(t.children[i, 0]),
                  int(n["rightChild"]) == int(t.children[i, 1]),
                  int(n["axis"]) == int(t.axis[i]),
                  (n["isLeftLeaf"] == "TRUE") == bool(t.is_leaf[i, 0]),
                  (n["isRightLeaf"] == "TRUE") == bool(t.is_leaf[i, 1]),
                  n["clipPlaneLEFT"] == "%g" % float(t.clip[i, 0]),
                  n["clipPlaneRIGHT"] == "%g" % float(t.clip[i, 1]))
        ok += all(fields)
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--write", action="store_true")
    args = ap.parse_args()
    exe = build_search()
    results = []
    winner = None
    for variant in (0, 1):
        for name, V, faces in vertex_sets(variant):
            inp = "\n".join(" ".join(float(x).hex() for x in row) for row in V.astype(np.float64))
            inp += "\n" + "\n".join(" ".join(str(i) for i in fc) for fc in faces) + "\n"
            r = subprocess.run([exe, DUMP], input=inp, capture_output=True, text=True, check=True)
            matches = [list(map(int, l.split()[1:])) for l in r.stdout.splitlines()
                       if l.startswith("MATCH")]
            summ = [l for l in r.stdout.splitlines() if l.startswith("SUMMARY")][0]
            rec = {"variant": variant, "precision": name, "summary": summ,
                   "matches": matches[:20], "n_matches": len(matches)}
            for m in matches:
                tris = soup(V, faces, m)
                rec.setdefault("oracle_nodes_matched", []).append(tree_matches_dump(tris))
                if winner is None and rec["oracle_nodes_matched"][-1] == 35:
                    winner = (variant, name, m, tris)
            print(json.dumps(rec), flush=True)
            results.append(rec)
    if winner is not None:
        print("WINNER", winner[:3])
        if args.write:
            np.save(OUT, winner[3])
            json.dump({"variant": winner[0], "precision": winner[1], "apex": winner[2],
                       "search": results}, open(META, "w"), indent=1)
    else:
        print("NO MATCH")
        if args.write:
            json.dump({"winner": None, "search": results}, open(META, "w"), indent=1)


if __name__ == "__main__":
    main()
