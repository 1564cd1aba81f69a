"""CPU checks of the map-maintenance oracle (oracle/map_oracle.cpp) on hand
cases of ikd-Tree's Add_Points rules (ikd_Tree.cpp:419-512) and of
lasermap_fov_segment (laserMapping.cpp:309-365).  The GPU mirror is held
to this oracle bit for bit in tests/test_gpu_map.py."""
import numpy as np


def dump(m):
    p, i = m.dump()
    return [tuple(v) for v in p], list(i)


def test_downsample_rules(oracle_mod):
    O = oracle_mod
    # box [0, 0.5)^3, centre (0.25, 0.25, 0.25)
    m = O.Map(np.array([[0.1, 0.1, 0.1]], np.float32))
    # a nearer new point replaces the single stored one (and gets id 1)
    assert m.add_points(np.array([[0.2, 0.24, 0.26]]), True, 0.5) == 1
    p, i = dump(m)
    assert i == [1] and np.allclose(p[0], (0.2, 0.24, 0.26))
    # a farther new point next to a single stored point: nothing happens
    assert m.add_points(np.array([[0.45, 0.45, 0.45]]), True, 0.5) == 0
    assert dump(m)[1] == [1]
    # a new point in an empty box is added
    assert m.add_points(np.array([[1.2, 0.1, 0.1]]), True, 0.5) == 1
    assert dump(m)[1] == [1, 2]


def test_downsample_many_stored(oracle_mod):
    O = oracle_mod
    pts = np.array([[0.05, 0.05, 0.05], [0.26, 0.24, 0.25], [0.45, 0.4, 0.4]], np.float32)
    m = O.Map(pts)
    # three stored points and a far new one: the box keeps only the stored
    # point nearest the centre (id 1), the new point is dropped
    assert m.add_points(np.array([[0.01, 0.49, 0.01]]), True, 0.5) == 1
    assert dump(m)[1] == [1]


def test_no_downsample_and_delete(oracle_mod):
    O = oracle_mod
    m = O.Map(np.zeros((0, 3), np.float32))
    pts = np.array([[0, 0, 0], [0, 0, 0], [1, 1, 1], [2, 2, 2]], np.float32)
    assert m.add_points(pts, False) == 0
    assert dump(m)[1] == [0, 1, 2, 3]
    # half-open boxes: [1, 2) keeps 2.0 out
    assert m.delete_boxes(np.array([[1, 1, 1, 2, 2, 2]], np.float32)) == 1
    assert dump(m)[1] == [0, 1, 3]
    assert m.delete_boxes(np.array([[-1, -1, -1, 0.5, 0.5, 0.5]], np.float32)) == 2
    assert dump(m)[1] == [3]


def test_fov_segment_moves(oracle_mod):
    lo, hi = np.zeros(3, np.float32), np.zeros(3, np.float32)
    ini, b = oracle_mod.fov_segment(np.zeros(3), lo, hi, False, cube_len=1000.0, det_range=300.0)
    assert ini and b.shape == (0, 6) and np.allclose(lo, -500) and np.allclose(hi, 500)
    # 60 m towards +x: 440 m from the max face <= 1.5 * 300 -> the box moves
    ini, b = oracle_mod.fov_segment(np.array([60.0, 0, 0]), lo, hi, ini, cube_len=1000.0, det_range=300.0)
    mov = max((1000 - 2 * 1.5 * 300) * 0.5 * 0.9, 300 * 0.5)
    assert b.shape == (1, 6) and np.allclose(b[0], [-500, -500, -500, -500 + mov, 500, 500])
    assert np.allclose(lo, [-500 + mov, -500, -500]) and np.allclose(hi, [500 + mov, 500, 500])
