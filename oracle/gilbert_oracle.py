"""TEST INFRASTRUCTURE ONLY — CPU restatement (oracle) of the Gilbert 3-D curve permutation.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker. The product computes the permutation in C++
(``video-blade_amd/csrc/vb_host.cpp``, exported as ``vb_gilbert3d_perm``).

Follows the generalized-Hilbert ("gilbert") curve of J. Cervený (BSD-2, 2018) as used by the
reference at ``cogvideox/train/special_attentions_local/utils/gilbert3d.py:6-167`` and the index
maps built in ``cogvideo_blocksparseattn.py:110-140`` (GilbertRearranger.__init__ /
_gilbert3d_with_index). Written as an explicit-stack traversal rather than a recursive generator;
the emitted point order is identical (pinned by ``tests/golden/gilbert_perms.npz``).

Parity: pinned against the reference's own generator run in this container
(``tests/golden/make_golden.py``) and against the reference's Gilbert test cases
(``cogvideox/sample_evaluate/Triton/tests/test_gilbert_rearranger.py:70-309``).
"""
from __future__ import annotations

import numpy as np


def _sgn(x: int) -> int:
    return (x > 0) - (x < 0)


def _l1(v):
    return abs(v[0] + v[1] + v[2])


def _add(*vs):
    return (sum(v[0] for v in vs), sum(v[1] for v in vs), sum(v[2] for v in vs))


def _neg(v):
    return (-v[0], -v[1], -v[2])


def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _half(v):
    # Python floor division on every component (negative components floor toward -inf).
    return (v[0] // 2, v[1] // 2, v[2] // 2)


def _unit(v):
    return (_sgn(v[0]), _sgn(v[1]), _sgn(v[2]))


def _children(p, a, b, c):
    """Split one box (origin p, major axis a, axes b, c) into ordered sub-boxes.

    Returns either ('line', start, step, n) for a 1-D run or ('split', [boxes...]).
    Follows generate3d (utils/gilbert3d.py:36-167)."""
    w, h, d = _l1(a), _l1(b), _l1(c)
    da, db, dc = _unit(a), _unit(b), _unit(c)
    if h == 1 and d == 1:
        return ("line", p, da, w)
    if w == 1 and d == 1:
        return ("line", p, db, h)
    if w == 1 and h == 1:
        return ("line", p, dc, d)
    a2, b2, c2 = _half(a), _half(b), _half(c)
    # prefer even sub-steps (gilbert3d.py:81-88)
    if (_l1(a2) % 2) and w > 2:
        a2 = _add(a2, da)
    if (_l1(b2) % 2) and h > 2:
        b2 = _add(b2, db)
    if (_l1(c2) % 2) and d > 2:
        c2 = _add(c2, dc)
    ra, rb, rc = _sub(a, a2), _sub(b, b2), _sub(c, c2)
    if 2 * w > 3 * h and 2 * w > 3 * d:          # wide: split a only (:90-99)
        return ("split", [(p, a2, b, c), (_add(p, a2), ra, b, c)])
    if 3 * h > 4 * d:                             # keep d whole (:101-116)
        return ("split", [
            (p, b2, c, a2),
            (_add(p, b2), a, rb, c),
            (_add(p, _sub(a, da), _sub(b2, db)), _neg(b2), c, _neg(ra)),
        ])
    if 3 * d > 4 * h:                             # keep h whole (:118-133)
        return ("split", [
            (p, c2, a2, b),
            (_add(p, c2), a, b, rc),
            (_add(p, _sub(a, da), _sub(c2, dc)), _neg(c2), _neg(ra), b),
        ])
    return ("split", [                            # regular 5-way split (:135-167)
        (p, b2, c2, a2),
        (_add(p, b2), c, a2, rb),
        (_add(p, _sub(b2, db), _sub(c, dc)), a, _neg(b2), _neg(rc)),
        (_add(p, _sub(a, da), b2, _sub(c, dc)), _neg(c), _neg(ra), rb),
        (_add(p, _sub(a, da), _sub(b2, db)), _neg(b2), c2, _neg(ra)),
    ])


def gilbert3d_points(width: int, height: int, depth: int):
    """Ordered list of (x, y, z) visiting every cell of a width×height×depth box once."""
    if width >= height and width >= depth:
        root = ((0, 0, 0), (width, 0, 0), (0, height, 0), (0, 0, depth))
    elif height >= width and height >= depth:
        root = ((0, 0, 0), (0, height, 0), (width, 0, 0), (0, 0, depth))
    else:
        root = ((0, 0, 0), (0, 0, depth), (width, 0, 0), (0, height, 0))
    pts = []
    stack = [root]
    while stack:
        kind, *rest = _children(*stack.pop())
        if kind == "line":
            start, step, n = rest
            x, y, z = start
            for _ in range(n):
                pts.append((x, y, z))
                x, y, z = x + step[0], y + step[1], z + step[2]
        else:
            stack.extend(reversed(rest[0]))
    return pts


def gilbert_perm(width: int, height: int, depth: int) -> np.ndarray:
    """perm[g] = linear index x + W*(y + H*z) of the g-th curve point.

    Equals ``GilbertRearranger.original_order2gilbert_order`` (cogvideo_blocksparseattn.py:119-127):
    rearranged[g] = original[perm[g]]."""
    pts = np.asarray(gilbert3d_points(width, height, depth), dtype=np.int64)
    return pts[:, 0] + width * (pts[:, 1] + height * pts[:, 2])


def inverse_perm(perm: np.ndarray) -> np.ndarray:
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size, dtype=perm.dtype)
    return inv


def full_sequence_perm(width: int, height: int, depth: int, text_length: int) -> np.ndarray:
    """Reordered position -> original token index for the whole [text | video] sequence.

    CogVideoX (text_length > 0, text FIRST in the input): reordered = [video[perm], text]
    (cogvideo_blocksparseattn.py:141-154). Wan (text_length == 0): reordered = x[perm]
    (wanx_blocksparseattn.py:142-152)."""
    perm = gilbert_perm(width, height, depth)
    return np.concatenate([perm + text_length, np.arange(text_length, dtype=np.int64)])
