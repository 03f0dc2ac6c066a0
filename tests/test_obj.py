"""OBJ scene ingestion: bih_scene_load_obj through the C ABI
against oracle/obj_oracle.py (restatement of assimp's fast_atof + OBJ
triangulation, reference src/Model.cpp:10-95, src/App.cpp:65-121,
src/assimp/fast_atof.h:259-344).  Host-only: no device is touched."""
import numpy as np
import pytest

F32 = np.float32


def _write(tmp_path, text, name="m.obj"):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def _load_both(bihrt_mod, tmp_path, text):
    import obj_oracle
    got = bihrt_mod.load_obj(_write(tmp_path, text))
    ref = obj_oracle.load_obj(text)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    return got


def test_triangle_and_convex_quad(bihrt_mod, tmp_path):
    text = "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf 1 2 3\nf 1 2 3 4\n"
    got = _load_both(bihrt_mod, tmp_path, text)
    v = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], F32)
    exp = np.stack([v[[0, 1, 2]].ravel(), v[[0, 1, 2]].ravel(), v[[0, 2, 3]].ravel()])
    assert np.array_equal(got, exp)


def test_concave_quad_fans_from_the_reflex_vertex(bihrt_mod, tmp_path):
    # dart: vertex 4 (index 3) is reflex; assimp fans (3,0,1), (3,1,2)
    text = "v 0 0 0\nv 2 1 0\nv 0 2 0\nv 0.5 1 0\nf 1 2 3 4\n"
    import obj_oracle
    pos = [[F32(0), F32(0), F32(0)], [F32(2), F32(1), F32(0)], [F32(0), F32(2), F32(0)],
           [F32(0.5), F32(1), F32(0)]]
    assert obj_oracle.quad_start(pos, [0, 1, 2, 3]) == 3
    got = _load_both(bihrt_mod, tmp_path, text)
    v = np.array(pos, F32)
    assert np.array_equal(got, np.stack([v[[3, 0, 1]].ravel(), v[[3, 1, 2]].ravel()]))


def test_obj_syntax_variants(bihrt_mod, tmp_path):
    text = "\n".join([
        "# comment line",
        "mtllib scene.mtl",
        "o first",
        "v 1.0 2.0 3.0",
        "v 4 5 6 2",               # homogeneous: (2, 2.5, 3)
        "v -1e-1 .5 7.",           # exponent, leading point, trailing point
        "v 1,5 2 3 0.1 0.2 0.3",   # comma decimal point, vertex colour ignored
        "vt 0 0",
        "vn 0 0 1",
        "g grp",
        "usemtl red",
        "s 1",
        "f 1/1/1 2/1/1 3/1/1",
        "usemtl blue",
        "f -4//1 -3//1 -1//1",     # relative indices
        "l 1 2",                   # line: dropped
        "p 3",                     # point: dropped
        "f 1 2",                   # two-index face: dropped
        "f 1 2 3 4 1/1",           # pentagon: fan from vertex 0
        "",
    ]) + "\r\n"
    got = _load_both(bihrt_mod, tmp_path, text)
    assert got.shape == (5, 9)
    assert np.array_equal(got[0, 3:6], np.array([2.0, 2.5, 3.0], F32))
    assert got[0, 6] == F32(-0.1) and got[0, 7] == F32(0.5) and got[0, 8] == F32(7.0)
    assert np.array_equal(got[1, 6:9], np.array([1.5, 2, 3], F32))


@pytest.mark.parametrize("text,line", [
    ("v 0 0 0\nv 1 0 0\nf 1 2 3\n", 3),            # out of range
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n", 4),   # index 0
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf -4 1 2\n", 4),  # relative before the start
    ("v 0 0\n", 1),                                # arity
    ("v 0 0 x\n", 1),                              # not a number
    ("v 1 2 3 0\n", 1),                            # w = 0
    ("v 1 2 3\nv 1 2 3\nv 1 2 3\nf a b c\n", 4),
])
def test_malformed_files_report_the_line(bihrt_mod, tmp_path, text, line):
    import obj_oracle
    with pytest.raises(bihrt_mod.BihError) as e:
        bihrt_mod.load_obj(_write(tmp_path, text))
    assert e.value.code == -9
    assert f"line {line}" in str(e.value)
    with pytest.raises(obj_oracle.ParseError) as e2:
        obj_oracle.load_obj(text)
    assert e2.value.line == line


def test_missing_file_is_io_error(bihrt_mod, tmp_path):
    with pytest.raises(bihrt_mod.BihError) as e:
        bihrt_mod.load_obj(str(tmp_path / "nope.obj"))
    assert e.value.code == -8


def test_empty_file_has_no_triangles(bihrt_mod, tmp_path):
    assert bihrt_mod.load_obj(_write(tmp_path, "# nothing\nv 1 2 3\n")).shape == (0, 9)


def test_fast_atof_known_answers():
    """fast_atoreal_move<float> is not a correctly rounded parser: these pin its
    arithmetic (integer part -> float, fraction as double -> float, added in
    float, exponent as powf)."""
    from obj_oracle import fast_atof
    assert fast_atof("1.5") == F32(1.5)
    assert fast_atof("-0.25") == F32(-0.25)
    assert fast_atof(".5") == F32(0.5) and fast_atof("7.") == F32(7.0)
    assert fast_atof("2,5") == F32(2.5)
    assert fast_atof("1e3") == F32(1000.0)
    # 16777217 -> float rounds to 16777216, and the fraction is added in float
    assert fast_atof("16777217.5") == F32(F32(16777216.0) + F32(0.5))
    # digits after the 15th fraction digit are ignored
    assert fast_atof("0.1234567890123459999") == F32(123456789012345 * 1e-15)
    # an integer part that overflows uint64 gives 0
    assert fast_atof("99999999999999999999.5") == F32(0.0)
    assert np.isnan(fast_atof("nan")) and fast_atof("-inf") == F32(-np.inf)


def test_fast_atof_fuzz_c_equals_python(bihrt_mod, tmp_path):
    """Random numeric spellings: the C loader and the Python restatement agree
    bit for bit on every coordinate."""
    rng = np.random.default_rng(11)
    toks = []
    for _ in range(3000):
        kind = rng.integers(0, 6)
        if kind == 0:
            toks.append(str(F32(rng.normal() * 10.0 ** rng.integers(-6, 7))))
        elif kind == 1:
            toks.append("%.*f" % (int(rng.integers(0, 20)), rng.uniform(-1e4, 1e4)))
        elif kind == 2:
            toks.append("%.*e" % (int(rng.integers(0, 12)), rng.normal() * 10.0 ** rng.integers(-30, 30)))
        elif kind == 3:
            toks.append(str(int(rng.integers(-2**40, 2**40))))
        elif kind == 4:
            toks.append("." + "".join(str(d) for d in rng.integers(0, 10, rng.integers(1, 25))))
        else:
            toks.append(repr(float(rng.uniform(-3, 3))))
    while len(toks) % 9:
        toks.append("0")
    lines = ["v %s %s %s" % tuple(toks[i:i + 3]) for i in range(0, len(toks), 3)]
    nv = len(lines)
    lines += ["f %d %d %d" % (i + 1, i + 2, i + 3) for i in range(0, nv, 3)]
    _load_both(bihrt_mod, tmp_path, "\n".join(lines) + "\n")


@pytest.mark.parametrize("shared", [False, True])
def test_round_trip_of_generated_scenes(bihrt_mod, tmp_path, shared):
    """Scenes written by bihrt.scenes.write_obj (shortest float32 repr) load
    back in file order, equal to the restatement, within one ulp of the soup
    (fast_atof is not correctly rounded)."""
    import obj_oracle
    from bihrt import scenes as S
    for name, tris in [("cornell", S.cornell()), ("torus", S.torus(40, 20)),
                       ("soup", S.soup(2000, seed=3))]:
        p = str(tmp_path / f"{name}.obj")
        S.write_obj(p, tris, shared=shared)
        got = bihrt_mod.load_obj(p)
        ref = obj_oracle.load_obj(open(p).read())
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), name
        t = np.asarray(tris, F32).reshape(-1, 9)
        ulp = np.abs(got.view(np.int32).astype(np.int64) - t.view(np.int32).astype(np.int64))
        assert got.shape == t.shape and int(ulp.max()) <= 1, name


def test_model_class(bihrt_mod, tmp_path):
    from bihrt import scenes as S
    p = str(tmp_path / "c.obj")
    S.write_obj(p, S.cornell())
    m = bihrt_mod.Model(p)
    assert len(m) == S.cornell().shape[0]
