"""ctypes binding of libgymchess.so (include/gymchess.h).

The shared library holds the HIP kernels for gfx950 and the extern "C" launch shim.
There is no CPU fallback: if the library is missing or no GPU is visible every call
fails loudly.
"""
import ctypes
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgymchess.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "gymchess.h")

# hipcc flags of libgymchess.so (__graft_entry__.build_hip); kernarg preload: the leading
# arguments of the step kernels arrive in SGPRs
BUILD_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
               "-mllvm", "-amdgpu-kernarg-preload-count=16"]
HASH_TAG = b"gymchess-src-hash:"


def source_hash():
    """sha256 prefix of the library's sources (csrc/*, include/gymchess.h) and BUILD_FLAGS, or
    None when the sources are not beside the package (an installed copy)"""
    if not os.path.isdir(CSRC) or not os.path.exists(HEADER):
        return None
    h = hashlib.sha256(" ".join(BUILD_FLAGS).encode())
    for p in sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)) + [HEADER]:
        if os.path.isfile(p):
            h.update(os.path.basename(p).encode() + b"\0")
            with open(p, "rb") as f:
                h.update(f.read())
    return h.hexdigest()[:16]


def built_hash(path=LIB_PATH):
    """the source hash embedded in a built library (gc_build_hash's string), read from the file"""
    with open(path, "rb") as f:
        data = f.read()
    k = data.find(HASH_TAG)
    if k < 0:
        return None
    return data[k + len(HASH_TAG): k + len(HASH_TAG) + 16].decode(errors="replace")

# every symbol declared in include/gymchess.h: name -> (restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
_U64 = ctypes.c_uint64
SIGNATURES = {
    "gc_last_error": (ctypes.c_char_p, []),
    "gc_version": (_I, []),
    "gc_build_hash": (ctypes.c_char_p, []),
    "gc_get_device_count": (_I, [_P]),
    "gc_engine_create": (_I, [_I, _P]),
    "gc_engine_destroy": (_I, [_P]),
    "gc_engine_get_possible_moves": (_I, [_P, _I, _P, _P, _P, _I, _P, _I, _P]),
    "gc_engine_get_castle_moves": (_I, [_P, _I, _P, _P, _P, _P, _P]),
    "gc_engine_next_state": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gc_engine_update_state": (_I, [_P, _I, _P, _P, _P, _P]),
    "gc_engine_perft": (_I, [_P, _I, _P, _P, _I, _P]),
    "gc_perft_path_counts": (_I, [_P]),
    "gc_perft_leaf_stats": (_I, [_P, _P, _P]),
    "gc_perft_dedup_stats": (_I, [_P, _P]),
    "gc_engine_set_rules": (_I, [_P, _I]),
    "gc_env_create": (_I, [_I, _I, _U64, _P, _P]),
    "gc_env_destroy": (_I, [_P]),
    "gc_env_set_opponent": (_I, [_P, _I, _I]),
    "gc_env_set_fens": (_I, [_P, _P]),
    "gc_fen_to_state": (_I, [ctypes.c_char_p, _P, _P]),
    "gc_state_to_fen": (_I, [_P, _P, _P, _I]),
    "gc_fen_to_state_rules": (_I, [ctypes.c_char_p, _P, _P, _I]),
    "gc_state_to_fen_rules": (_I, [_P, _P, _P, _I, _I]),
    "gc_env_set_rules": (_I, [_P, _I]),
    "gc_env_num_boards": (_I, [_P]),
    "gc_env_reset": (_I, [_P, _P]),
    "gc_env_step": (_I, [_P, _P, _P, _P, _P]),
    "gc_env_step_random": (_I, [_P, _I]),
    "gc_env_select_random": (_I, [_P]),
    "gc_env_set_streams": (_I, [_P, _I]),
    "gc_env_paired": (_I, [_P]),
    "gc_env_rollout_waves": (_I, [_P]),
    "gc_env_rollout_occ_min_plies": (_I, []),
    "gc_env_step_device": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I]),
    "gc_env_step_device2": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, ctypes.c_int64]),
    "gc_env_get_stream": (_I, [_P, _P]),
    "gc_device_alloc": (_I, [_I, _U64, _P]),
    "gc_device_free": (_I, [_I, _P]),
    "gc_env_copy": (_I, [_P, _P, _P, _U64, _I]),
    "gc_env_rollout": (_I, [_P, _I, _P, _P, _P, _P, _P]),
    "gc_env_rollout_device": (_I, [_P, _I, _P, _I, _I]),
    "gc_env_spill_info": (_I, [_P, _P, _P, _P]),
    "gc_env_single_setup": (_I, [_P, _I]),
    "gc_env_single_call": (_I, [_P, _I, _I, _I, _I, _P]),
    "gc_env_single_set": (_I, [_P, _I, _P, _P, _P]),
    "gc_env_single_stamps": (_I, [_P, _P]),
    "gc_env_window_boards": (_I, [_P, _I, _P, _P, _I, _P]),
    "gc_env_get_outputs": (_I, [_P, _P, _P, _P, _P, _P]),
    "gc_env_get_states": (_I, [_P, _P, _P]),
    "gc_env_set_states": (_I, [_P, _P, _P]),
    "gc_env_legal_moves": (_I, [_P, _P, _I, _P]),
    "gc_env_legal_mask": (_I, [_P, _P, _P]),
    "gc_env_synchronize": (_I, [_P]),
    "gc_env_wait_rollout": (_I, [_P]),
    "gc_env_record_event": (_I, [_P, _I]),
    "gc_env_elapsed_ms": (_I, [_P, _I, _I, _P]),
    "gc_env_device_bytes": (_U64, [_P]),
    "gc_env_window_sum": (_I, [_P, _P]),
    "gc_env_checkpoint_bytes": (_I, [_P, _P]),
    "gc_env_get_en_passant": (_I, [_P, _P]),
    "gc_env_set_en_passant": (_I, [_P, _P]),
    "gc_env_save": (_I, [_P, _P, _U64, _P]),
    "gc_env_load": (_I, [_P, _P, _U64]),
}

_lib = None


class GymChessError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load libgymchess.so (raises if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GymChessError(
            f"{path} not found: the HIP extension is not built (python -c 'import __graft_entry__ as g; g.build()')"
        )
    if path == LIB_PATH and os.environ.get("GC_ALLOW_STALE_LIB") != "1":
        want = source_hash()
        if want is not None and built_hash(path) != want:
            raise GymChessError(
                f"{path} was built from other sources (hash {built_hash(path)}, sources {want}): rebuild it "
                "(python -c 'import __graft_entry__ as g; g.build()')"
            )
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


RULES = {"reference": 0, "fide": 1}


def rules_id(rules):
    """'reference' (default: lib.rs's rules) or 'fide' (gc_fide.h) -> the C-ABI's rules code."""
    if rules not in RULES:
        raise ValueError(f"rules must be one of {sorted(RULES)}, got {rules!r}")
    return RULES[rules]


def check(rc):
    if rc != 0:
        msg = load().gc_last_error()
        raise GymChessError(msg.decode() if msg else f"gymchess call failed ({rc})")


def ptr(a):
    """numpy array -> its data address for a void* argument (the array must stay alive for the
    call; an int converts at the call, ~5x cheaper than ctypes.data_as)."""
    return a.ctypes.data


def device_count():
    n = ctypes.c_int(0)
    check(load().gc_get_device_count(ctypes.byref(n)))
    return n.value
