"""ctypes binding of libhuygens_hip.so (the C ABI declared in include/huygens_hip.h).

The product path has no CPU fallback: if the HIP library is missing or no gfx950
device is visible, every call raises HZError.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HZ_LIB_PATH") or os.path.join(_HERE, "lib", "libhuygens_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "huygens_hip.h")

HZ_OK = 0
HZ_E_INVALID = -1
HZ_E_RANGE = -2
HZ_E_HIP = -3
HZ_E_NODEV = -4
HZ_E_ALLOC = -5
HZ_E_UNSUPPORTED = -6
HZ_E_STATE = -7

HZ_FB_PATH_AUTO = 0
HZ_FB_PATH_GENERAL = 1
HZ_FB_PATH_LTI = 2
HZ_FB_PATH_RESPONSE = 3
HZ_FB_PATH_STREAM = 4

HZ_FB_RESP_OFF = 0
HZ_FB_RESP_EAGER = 1
HZ_FB_RESP_LAZY = 2

HZ_DIST_NONE = 0
HZ_DIST_SOFTCLIP = 1
HZ_DIST_SATURATE = 2
HZ_DIST_LIMITER = 3

_ERRNAMES = {
    HZ_E_INVALID: "HZ_E_INVALID", HZ_E_RANGE: "HZ_E_RANGE", HZ_E_HIP: "HZ_E_HIP",
    HZ_E_NODEV: "HZ_E_NODEV", HZ_E_ALLOC: "HZ_E_ALLOC", HZ_E_UNSUPPORTED: "HZ_E_UNSUPPORTED",
    HZ_E_STATE: "HZ_E_STATE",
}


class HZError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


_lib = None

D = C.c_double
I = C.c_int
L = C.c_long
SZ = C.c_size_t
VP = C.c_void_p
PD = C.POINTER(C.c_double)

# name -> (restype, argtypes)
_SIGS = {
    "hz_last_error": (C.c_char_p, []),
    "hz_version": (I, []),
    "hz_device_count": (I, []),
    # Filterbank
    "hz_fb_create": (I, [I, I, D, D, I, C.POINTER(VP)]),
    "hz_fb_create_shard": (I, [I, I, I, I, D, D, I, C.POINTER(VP)]),
    "hz_fb_destroy": (I, [VP]),
    "hz_fb_coefficients": (I, [VP, I, PD, I, PD, I]),
    "hz_fb_boost": (I, [VP, I, D]),
    "hz_fb_boost_all": (I, [VP, PD, I]),
    "hz_fb_mix": (I, [VP, I, D]),
    "hz_fb_mix_all": (I, [VP, PD, I]),
    "hz_fb_open": (I, [VP]),
    "hz_fb_set_distortion": (I, [VP, I, D]),
    "hz_fb_process": (I, [VP, PD, PD, SZ]),
    "hz_fb_process_device": (I, [VP, VP, VP, SZ]),
    "hz_fb_tick": (I, [VP]),
    "hz_fb_sample": (I, [VP, D, I, D, PD]),
    "hz_fb_sample_tick": (I, [VP]),
    "hz_fb_sample_info": (I, [VP, C.POINTER(I), C.POINTER(C.c_longlong), C.POINTER(I)]),
    "hz_fb_process_tv": (I, [VP, PD, PD, SZ, I, PD, D]),
    "hz_fb_process_tv_device": (I, [VP, VP, VP, SZ, I, VP, D]),
    "hz_fb_set_stream": (I, [VP, VP]),
    "hz_fb_get_stream": (I, [VP, C.POINTER(VP)]),
    "hz_fb_synchronize": (I, [VP]),
    "hz_fb_state_size": (I, [VP, C.POINTER(SZ)]),
    "hz_fb_get_state": (I, [VP, PD, SZ]),
    "hz_fb_set_state": (I, [VP, PD, SZ]),
    "hz_fb_info": (I, [VP, C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "hz_fb_tune": (I, [VP, I, I]),
    "hz_fb_profile": (I, [VP, I]),
    "hz_fb_profile_read": (I, [VP, PD, PD, PD, C.POINTER(L)]),
    "hz_fb_set_target_groups": (I, [VP, I]),
    "hz_fb_set_path": (I, [VP, I]),
    "hz_fb_last_path": (I, [VP, C.POINTER(I)]),
    "hz_fb_tune_lti": (I, [VP, I, I, I]),
    "hz_fb_lti_plan": (I, [VP, C.POINTER(C.c_long), C.POINTER(C.c_long), C.POINTER(C.c_int)]),
    "hz_fb_lti_last_chunk": (I, [VP, C.POINTER(C.c_int)]),
    "hz_fb_set_response": (I, [VP, I]),
    "hz_fb_tune_response": (I, [VP, L, L]),
    "hz_fb_tune_response_engine": (I, [VP, I]),
    "hz_fb_sample_many": (I, [C.POINTER(VP), I, PD, I, D, PD]),
    "hz_fb_response_engine": (I, [VP, C.POINTER(I), C.POINTER(I)]),
    "hz_fb_tune_modal": (I, [VP, I]),
    "hz_fb_modal_info": (I, [VP, C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "hz_fb_response_info": (I, [VP, C.POINTER(L), C.POINTER(L), C.POINTER(I), C.POINTER(L)]),
    "hz_fb_get_response": (I, [VP, PD, L]),
    "hz_fb_set_bank_response": (I, [VP, PD, L]),
    "hz_fb_set_time_shard": (I, [VP, I, I]),
    "hz_fb_set_time_shard_fill": (I, [VP, I]),
    "hz_fb_time_shard_info": (I, [VP, C.POINTER(I), C.POINTER(L), C.POINTER(L), L]),
    "hz_fb_stationary_ready": (I, [VP, L, C.POINTER(I)]),
    "hz_fb_arm_time_shard": (I, [VP, I]),
    "hz_fb_tune_stream": (I, [VP, I]),
    "hz_fb_setter_seq": (I, [VP, C.POINTER(C.c_longlong)]),
    "hz_dly_sample": (I, [VP, VP, VP, I]),
    "hz_gran_sample": (I, [VP, D, PD]),
    "hz_rt_info": (I, [I, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong), C.POINTER(I)]),
    "hz_add_lookahead_info": (I, [VP, C.POINTER(L), C.POINTER(L), C.POINTER(L)]),
    "hz_fb_stream_info": (I, [VP, C.POINTER(I), C.POINTER(L), C.POINTER(L), C.POINTER(I)]),
    # Oscbank
    "hz_osc_create": (I, [I, D, I, C.POINTER(VP)]),
    "hz_osc_create_shard": (I, [I, I, I, D, I, C.POINTER(VP)]),
    "hz_osc_destroy": (I, [VP]),
    "hz_osc_freqmod": (I, [VP, I, D]),
    "hz_osc_activate": (I, [VP, C.POINTER(I), I]),
    "hz_osc_deactivate": (I, [VP, C.POINTER(I), I]),
    "hz_osc_open": (I, [VP]),
    "hz_osc_close": (I, [VP]),
    "hz_osc_active_count": (I, [VP, C.POINTER(I)]),
    "hz_osc_fill": (I, [VP, PD, PD, SZ]),
    "hz_osc_fill_device": (I, [VP, VP, VP, SZ]),
    "hz_osc_mixdown": (I, [VP, PD]),
    "hz_osc_phases": (I, [VP, PD]),
    "hz_osc_set_phases": (I, [VP, PD]),
    "hz_osc_set_stream": (I, [VP, VP]),
    "hz_osc_synchronize": (I, [VP]),
    "hz_osc_set_target_groups": (I, [VP, I]),
    "hz_osc_profile": (I, [VP, I]),
    "hz_osc_profile_read": (I, [VP, PD, C.POINTER(L)]),
    # Additive / Sinusoids
    "hz_add_create": (I, [I, I, D, D, D, I, C.POINTER(VP)]),
    "hz_add_create_shard": (I, [I, I, I, I, D, D, D, I, C.POINTER(VP)]),
    "hz_add_destroy": (I, [VP]),
    "hz_add_request": (I, [VP, D, D, C.POINTER(I)]),
    "hz_add_release": (I, [VP, I]),
    "hz_add_makenote": (I, [VP, D, D, C.POINTER(I)]),
    "hz_add_endnote": (I, [VP, D]),
    "hz_add_fill": (I, [VP, PD, SZ]),
    "hz_add_fill_device": (I, [VP, VP, SZ]),
    "hz_add_set_stream": (I, [VP, VP]),
    "hz_add_set_target_groups": (I, [VP, I]),
    "hz_add_profile": (I, [VP, I]),
    "hz_add_profile_read": (I, [VP, PD, C.POINTER(L)]),
    "hz_sin_create": (I, [D, I, D, D, D, I, C.POINTER(VP)]),
    "hz_sin_destroy": (I, [VP]),
    "hz_sin_fundmod": (I, [VP, D]),
    "hz_sin_decaymod": (I, [VP, D]),
    "hz_sin_harmmod": (I, [VP, D]),
    "hz_sin_fill": (I, [VP, PD, SZ]),
    "hz_sin_fill_device": (I, [VP, VP, SZ]),
    # Bowl
    "hz_bowl_create": (I, [I, PD, PD, PD, I, I, I, C.POINTER(VP)]),
    "hz_bowl_destroy": (I, [VP]),
    "hz_bowl_trigger": (I, [VP]),
    "hz_bowl_fill": (I, [VP, C.POINTER(C.c_float), SZ]),
    "hz_bowl_fill_device": (I, [VP, VP, SZ]),
    "hz_bowl_render": (I, [VP, PD, SZ]),
    "hz_bowl_render_device": (I, [VP, VP, SZ]),
    "hz_bowl_phase": (I, [VP, PD]),
    "hz_bowl_set_stream": (I, [VP, VP]),
    "hz_bowl_set_target_groups": (I, [VP, I]),
    "hz_bowl_profile": (I, [VP, I]),
    "hz_bowl_profile_read": (I, [VP, PD, C.POINTER(L)]),
    "hz_bowl_fill_delaybank": (I, [VP, VP, VP, VP, SZ, I]),
    "hz_dly_create": (I, [I, C.c_uint, C.c_uint, I, I, C.POINTER(VP)]),
    "hz_dly_destroy": (I, [VP]),
    "hz_dly_coefficients": (I, [VP, I, C.POINTER(C.c_uint), PD, I, C.POINTER(C.c_uint), PD, I]),
    "hz_dly_modulate_forward": (I, [VP, I, C.c_uint, C.c_uint, D]),
    "hz_dly_modulate_back": (I, [VP, I, C.c_uint, C.c_uint, D]),
    "hz_dly_process": (I, [VP, VP, VP, SZ, I, I]),
    "hz_dly_process_device": (I, [VP, VP, VP, SZ, I, I]),
    "hz_dly_tick": (I, [VP, C.c_ulong]),
    "hz_dly_origin": (I, [VP, C.POINTER(C.c_uint)]),
    "hz_dly_info": (I, [VP, C.POINTER(L), C.POINTER(C.c_uint)]),
    "hz_dly_set_split": (I, [VP, I]),
    "hz_dly_set_stream": (I, [VP, VP]),
    "hz_dly_synchronize": (I, [VP]),
    "hz_dly_set_target_groups": (I, [VP, I]),
    "hz_dly_profile": (I, [VP, I]),
    "hz_dly_profile_read": (I, [VP, PD, C.POINTER(L)]),
    "hz_stft_create": (I, [I, I, I, I, D, D, I, C.POINTER(VP)]),
    "hz_stft_destroy": (I, [VP]),
    "hz_stft_set_processor": (I, [VP, VP]),
    "hz_stft_process_block": (I, [VP, PD, PD, PD, PD, SZ]),
    "hz_stft_process_block_device": (I, [VP, VP, VP, VP, VP, SZ]),
    "hz_stft_frames": (I, [VP, C.POINTER(L), C.POINTER(L)]),
    "hz_stft_write": (I, [VP, D, D]),
    "hz_stft_read": (I, [VP, PD, PD]),
    "hz_stft_forward": (I, [VP, I]),
    "hz_stft_backward": (I, [VP, I]),
    "hz_stft_process_slot": (I, [VP, I]),
    "hz_stft_set_frame_shard": (I, [VP, I, I, C.c_long]),
    "hz_stft_frames_before": (I, [I, I, C.c_long, C.POINTER(C.c_long)]),
    "hz_stft_set_stream": (I, [VP, VP]),
    "hz_stft_synchronize": (I, [VP]),
    "hz_stft_profile": (I, [VP, I]),
    "hz_stft_profile_read": (I, [VP, PD, PD, C.POINTER(L)]),
    "hz_dct_create": (I, [I, I, C.POINTER(VP)]),
    "hz_dct_destroy": (I, [VP]),
    "hz_dct_buffers": (I, [VP, C.POINTER(PD), C.POINTER(PD)]),
    "hz_dct_forward": (I, [VP]),
    "hz_dct_backward": (I, [VP]),
    "hz_dct_forward_device": (I, [VP, VP, VP, I]),
    "hz_dct_backward_device": (I, [VP, VP, VP, I]),
    # Granulator
    "hz_gran_create": (I, [C.c_uint, C.c_uint, I, C.POINTER(VP)]),
    "hz_gran_destroy": (I, [VP]),
    "hz_gran_request": (I, [VP, D, D, D, D, D, I, C.POINTER(I)]),
    "hz_gran_process": (I, [VP, PD, PD, SZ, VP, I, C.POINTER(I)]),
    "hz_gran_process_device": (I, [VP, VP, VP, SZ, VP, I, C.POINTER(I)]),
    "hz_gran_activity": (I, [VP, C.POINTER(C.c_uint)]),
    "hz_gran_set_stream": (I, [VP, VP]),
    "hz_gran_synchronize": (I, [VP]),
    "hz_gran_profile": (I, [VP, I]),
    "hz_gran_profile_read": (I, [VP, PD, C.POINTER(L), C.POINTER(L)]),
    # heterodyne chain
    "hz_het_create": (I, [I, I, PD, D, D, C.c_uint, I, D, D, D, I, C.POINTER(VP)]),
    "hz_het_destroy": (I, [VP]),
    "hz_het_setup": (I, [VP, I, PD]),
    "hz_het_freqmod": (I, [VP, I, C.POINTER(I), PD, I]),
    "hz_het_activate": (I, [VP, I, C.POINTER(I), I, I]),
    "hz_het_open": (I, [VP, I, I]),
    "hz_het_process": (I, [VP, PD, PD, SZ]),
    "hz_het_process_device": (I, [VP, VP, VP, SZ]),
    "hz_het_state": (I, [VP, I, PD]),
    "hz_het_set_stream": (I, [VP, VP]),
    "hz_het_synchronize": (I, [VP]),
    "hz_het_profile": (I, [VP, I]),
    "hz_het_profile_read": (I, [VP, PD, C.POINTER(L), C.POINTER(L)]),
    # Freezer
    "hz_frz_create": (I, [I, I, D, I, C.POINTER(VP)]),
    "hz_frz_destroy": (I, [VP]),
    "hz_frz_freeze": (I, [VP]),
    "hz_frz_unfreeze": (I, [VP]),
    "hz_frz_process": (I, [VP, PD, PD, SZ, VP, I]),
    "hz_frz_process_device": (I, [VP, VP, VP, SZ, VP, I]),
    "hz_frz_info": (I, [VP, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "hz_frz_set_stream": (I, [VP, VP]),
    "hz_frz_synchronize": (I, [VP]),
    "hz_frz_profile": (I, [VP, I]),
    "hz_frz_profile_read": (I, [VP, C.POINTER(C.c_double), C.POINTER(C.c_long)]),
}


def load():
    """Load (once) and return the ctypes library; raises HZError when absent."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch-ROCm ships its own libamdhip64.so.7
    # (same SONAME as /opt/rocm's).  Whichever loads first serves both, and
    # torch refuses to initialise on top of the newer system runtime, so let
    # torch (when installed) load first.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise HZError(HZ_E_UNSUPPORTED, f"{LIB_PATH} not built (run `make lib` or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def header_symbols(path: str = HEADER_PATH):
    """Every hz_* function declared in include/huygens_hip.h."""
    txt = open(path).read()
    return sorted(set(re.findall(r"\b(hz_[a-z0-9_]+)\s*\(", txt)))


def check(code: int):
    if code != HZ_OK:
        msg = load().hz_last_error()
        raise HZError(code, msg.decode() if msg else "")
    return code


def dptr(a):
    """ctypes double* of a C-contiguous float64 numpy array."""
    return a.ctypes.data_as(PD)


def rt_info(device: int = 0):
    """The per-sample server (hz_rt.hip) of a device: (requests served, kernel launches, resident)."""
    lib = load()
    r, n, a = C.c_longlong(), C.c_longlong(), C.c_int()
    check(lib.hz_rt_info(device, C.byref(r), C.byref(n), C.byref(a)))
    return r.value, n.value, bool(a.value)
