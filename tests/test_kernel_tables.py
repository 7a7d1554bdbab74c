"""CPU checks of the constant tables baked into csrc/kernels/convnet.hip: the m-tile -> position maps
of the conv2 forward / dgrad kernels must be permutations of the output positions (padding = 255), and
the LDS bank model they were generated with must report the conflict-free schedule they promise."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def table(name):
    src = open(os.path.join(ROOT, "csrc", "kernels", "convnet.hip")).read()
    m = re.search(r"__constant__ uint8_t %s\[(\d+)\] = \{([^}]*)\};" % name, src)
    assert m, name
    vals = [int(v) for v in m.group(2).split(",")]
    assert len(vals) == int(m.group(1))
    return vals


@pytest.mark.parametrize("name,npos,ntiles", [("c2f_tile_pos", 121, 8), ("c2d_tile_pos", 169, 11)])
def test_tile_maps_are_permutations(name, npos, ntiles):
    t = table(name)
    assert len(t) == 16 * ntiles
    real = [v for v in t if v != 255]
    assert sorted(real) == list(range(npos))


@pytest.mark.parametrize("name,pw,width,stride", [("c2f_tile_pos", 13, 11, 48), ("c2d_tile_pos", 15, 13, 80)])
def test_full_tiles_are_residue_balanced(name, pw, width, stride):
    """Every full tile: lanes {0-3,12-15} and lanes {4-11} each hold 8 distinct residues (y*pw + x) mod 8,
    which with rows of `stride` bf16 (an odd multiple of 32 B) puts a ds_read_b128 lane group on 16
    distinct 16-B bank slots."""
    assert (stride * 2 // 32) % 2 == 1
    t = table(name)
    groups = ([0, 1, 2, 3, 12, 13, 14, 15], list(range(4, 12)))
    full = 0
    for k in range(len(t) // 16):
        tile = t[16 * k:16 * k + 16]
        if 255 in tile:
            continue
        full += 1
        for g in groups:
            res = {((tile[l] // width) * pw + tile[l] % width) % 8 for l in g}
            assert len(res) == 8, (name, k)
    assert full >= len(t) // 16 - 1
