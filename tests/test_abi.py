"""CPU checks of the boundary: libgymchess.so loads without a GPU, exports every symbol
include/gymchess.h declares, and the pure-Python host codecs follow the reference."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "gymchess.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    so = os.path.join(ROOT, "gym-chess_amd", "gym_chess_amd", "libgymchess.so")
    if not os.path.exists(so):
        import __graft_entry__ as g

        g.build_hip()
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gc_\w+)", out))
    declared = header_symbols()
    assert len(declared) >= 25
    missing = [s for s in declared if s not in exported]
    assert not missing, missing


def test_ctypes_binding_covers_header():
    from gym_chess_amd import _lib

    assert sorted(_lib.SIGNATURES) == header_symbols()
    L = _lib.load()  # loads without a GPU; resolves every symbol
    assert L.gc_version() == 1
    # the library is the build of the sources beside it (content hash, not mtimes)
    assert L.gc_build_hash().decode() == "gymchess-src-hash:" + _lib.source_hash()


def test_loader_refuses_a_library_from_other_sources(tmp_path):
    """A stale libgymchess.so (its embedded source hash differs from the sources') fails
    loudly at load instead of being tested silently (in a child process: the loader caches)."""
    import sys

    from gym_chess_amd import _lib

    stale = tmp_path / "libgymchess.so"
    data = open(_lib.LIB_PATH, "rb").read()
    k = data.find(_lib.HASH_TAG) + len(_lib.HASH_TAG)
    stale.write_bytes(data[:k] + b"0" * 16 + data[k + 16:])
    code = (f"import sys; sys.path.insert(0, {os.path.join(ROOT, 'gym-chess_amd')!r})\n"
            "from gym_chess_amd import _lib\n"
            f"_lib.LIB_PATH = {str(stale)!r}\n"
            "try:\n    _lib.load(_lib.LIB_PATH)\nexcept _lib.GymChessError as e:\n    print('refused', e)\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout
    assert out.startswith("refused") and "other sources" in out, out


def test_product_has_no_oracle_dependency():
    """The shipped package must not import or link the oracle (no CPU fallback)."""
    pkg = os.path.join(ROOT, "gym-chess_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "gcoracle" not in txt and "oracle_" not in txt, f


def test_no_gpu_raises_loudly():
    import ctypes

    from gym_chess_amd import _lib

    n = ctypes.c_int(-1)
    rc = _lib.load().gc_get_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    from gym_chess_amd.engine import Engine

    with pytest.raises(_lib.GymChessError):
        Engine(0)


def test_codec_roundtrip():
    from gym_chess_amd import codec as C

    for a in range(4096):
        s = C.action_to_str(a)
        assert C.str_to_action(s) == a
        assert C.move_to_action(C.action_to_move(a)) == a
        assert C.move_to_action(C.rust_move_to_coords(s)) == a
    assert C.action_to_str(52 * 64 + 36) == "e2e4"
    for name, a in C.CASTLE_TO_ACTION.items():
        assert C.action_to_str(a) == name and C.str_to_action(name) == a
    assert C.move_to_action(C.RESIGN) == 4100


def test_state_dict_roundtrip():
    from gym_chess_amd import codec as C

    st = dict(board=C.DEFAULT_BOARD, current_player="BLACK", white_king_castle_is_possible=True,
              white_queen_castle_is_possible=False, black_king_castle_is_possible=True,
              black_queen_castle_is_possible=False)
    b, m = C.dict_to_arrays(st)
    assert list(m[:5]) == [0, 1, 0, 1, 0]
    d = C.arrays_to_dict(b, m)
    assert d["board"] == C.DEFAULT_BOARD and d["current_player"] == "BLACK"
    with pytest.raises(KeyError):
        C.dict_to_arrays({"board": C.DEFAULT_BOARD})
    with pytest.raises(ValueError):
        C.player_to_white("GREEN")
    bad = dict(st, board=np.full((8, 8), 9))
    with pytest.raises(ValueError):
        C.dict_to_arrays(bad)
    assert C.board_to_text(C.text_to_board("K" + "." * 62 + "k")) == "K" + "." * 62 + "k"
