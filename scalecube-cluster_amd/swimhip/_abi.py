"""ctypes mirror of include/swimhip.h (the C ABI of libswimhip).

The same ABI is exported by the product library (libswimhip.so, gfx950) and, for tests only, by the CPU oracle
(oracle/liboracle_swimref.so). This module only describes the ABI. Choosing a library is the caller's job.
"""
import ctypes as C

SWIM_OK = 0
SWIM_EINVAL = -1
SWIM_ENOMEM = -2
SWIM_EDEVICE = -3
SWIM_ECAPACITY = -4
SWIM_EUNSUPPORTED = -5

INIT_COLD_JOIN = 0
INIT_PRECONVERGED = 1
MODE_FULL, MODE_RUMOR = 0, 1
FLAG_RECORD_EVENTS = 1
FLAG_PROFILE = 2
FLAG_PROFILE_ALL = 4
FLAG_IMPLICIT_VIEWS = 8
FLAG_EMULATOR_COUNTERS = 16

EV_ADDED, EV_REMOVED, EV_UPDATED, EV_GOSSIP = 0, 1, 2, 3
META_NONE = 0xFFFFFFFF
ST_ABSENT, ST_ALIVE, ST_SUSPECT, ST_DEAD = 0, 1, 2, 3
HASH_WORDS = 6  # row, fd list, gossip list, events, gossips held, misc


class SwimConfig(C.Structure):
    _fields_ = [
        ("n_members", C.c_uint32),
        ("tick_ms", C.c_uint32),
        ("latency_ticks", C.c_uint32),
        ("init_mode", C.c_uint32),
        ("seed", C.c_uint64),
        ("sync_interval_ms", C.c_uint32),
        ("sync_timeout_ms", C.c_uint32),
        ("suspicion_mult", C.c_uint32),
        ("ping_interval_ms", C.c_uint32),
        ("ping_timeout_ms", C.c_uint32),
        ("ping_req_members", C.c_uint32),
        ("gossip_interval_ms", C.c_uint32),
        ("gossip_fanout", C.c_uint32),
        ("gossip_repeat_mult", C.c_uint32),
        ("metadata_timeout_ms", C.c_uint32),
        ("mode", C.c_uint32),
        ("flags", C.c_uint32),
        ("n_seeds", C.c_uint32),
        ("seeds", C.c_uint32 * 16),
        ("gossip_slot_cap", C.c_uint32),
        ("pending_fetch_cap", C.c_uint32),
        ("event_cap", C.c_uint32),
        ("n_gpus", C.c_uint32),
        ("device", C.c_uint32),
        ("list_slack", C.c_uint32),
        ("churn_per_period", C.c_uint32),
        ("n_dormant", C.c_uint32),
        ("gossip_ring_cap", C.c_uint32),
        ("delay_cap_ms", C.c_uint32),
        ("reserved", C.c_uint32 * 2),
    ]


class SwimMemberConfig(C.Structure):
    _fields_ = [
        ("ping_interval_ms", C.c_uint32),
        ("ping_timeout_ms", C.c_uint32),
        ("ping_req_members", C.c_uint32),
        ("sync_group", C.c_uint32),
        ("reserved", C.c_uint32 * 4),
    ]


class SwimEvent(C.Structure):
    _fields_ = [
        ("tick", C.c_uint32),
        ("observer", C.c_uint32),
        ("seq", C.c_uint32),
        ("type", C.c_uint32),
        ("subject", C.c_uint32),
        ("old_meta", C.c_uint32),
        ("new_meta", C.c_uint32),
        ("pad", C.c_uint32),
    ]


class SwimCounters(C.Structure):
    _fields_ = [
        ("tick", C.c_uint64),
        ("record_compares", C.c_uint64),
        ("row_writes", C.c_uint64),
        ("messages", C.c_uint64),
        ("gossip_messages", C.c_uint64),
        ("events", C.c_uint64),
        ("messages_lost", C.c_uint64),
        ("gossips_created", C.c_uint64),
        ("sync_merges", C.c_uint64),
        ("device_bytes", C.c_uint64),
        ("diff_ns", C.c_uint64),
        ("member_ns", C.c_uint64),
        ("gossip_ns", C.c_uint64),
        ("diff_launches", C.c_uint64),
        ("exchange_ns", C.c_uint64),
        ("diff_msgs", C.c_uint64),
        ("ack_resolved", C.c_uint64),
        ("ack_resolved_total", C.c_uint64),
        ("diff_msgs_total", C.c_uint64),
        ("diff_key_bytes", C.c_uint64),
        ("diff_key_bytes_total", C.c_uint64),
    ]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_ if k != "reserved"}


# every entry point declared in include/swimhip.h: name -> (restype, argtypes)
_H = C.c_void_p
_U32P = C.POINTER(C.c_uint32)
SIGNATURES = {
    "swim_default_config": (None, [C.POINTER(SwimConfig)]),
    "swim_abi_version": (C.c_uint32, []),
    "swim_create": (C.c_int, [C.POINTER(SwimConfig), C.POINTER(_H)]),
    "swim_destroy": (C.c_int, [_H]),
    "swim_step": (C.c_int, [_H, C.c_uint32]),
    "swim_run_periods": (C.c_int, [_H, C.c_uint32]),
    "swim_sync": (C.c_int, [_H]),
    "swim_kill": (C.c_int, [_H, C.c_uint32]),
    "swim_set_default_loss": (C.c_int, [_H, C.c_uint32]),
    "swim_set_partition": (C.c_int, [_H, _U32P]),
    "swim_unblock_all": (C.c_int, [_H]),
    "swim_set_link_loss": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32]),
    "swim_set_default_link_settings": (C.c_int, [_H, C.c_uint32, C.c_uint32]),
    "swim_set_link_settings": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "swim_emulator_counters": (C.c_int, [_H, C.POINTER(C.c_uint64), C.c_size_t]),
    "swim_unblock_link": (C.c_int, [_H, C.c_uint32, C.c_uint32]),
    "swim_update_incarnation": (C.c_int, [_H, C.c_uint32]),
    "swim_update_metadata": (C.c_int, [_H, C.c_uint32]),
    "swim_leave": (C.c_int, [_H, C.c_uint32]),
    "swim_spread_gossip": (C.c_int, [_H, C.c_uint32, C.c_uint64]),
    "swim_join": (C.c_int, [_H, C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32]),
    "swim_set_member_config": (C.c_int, [_H, C.c_uint32, C.POINTER(SwimMemberConfig)]),
    "swim_current_tick": (C.c_int, [_H, C.POINTER(C.c_uint64)]),
    "swim_read_row": (C.c_int, [_H, C.c_uint32, C.POINTER(C.c_uint64), C.c_size_t]),
    "swim_state_hash": (C.c_int, [_H, C.POINTER(C.c_uint64), C.c_size_t]),
    "swim_read_lists": (C.c_int, [_H, C.c_uint32, _U32P, _U32P, _U32P, _U32P, C.c_size_t, C.POINTER(C.c_int32)]),
    "swim_read_gossips": (C.c_int, [_H, C.c_uint32, C.POINTER(C.c_uint64), _U32P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "swim_drain_events": (C.c_int, [_H, C.POINTER(SwimEvent), C.c_size_t, C.POINTER(C.c_size_t)]),
    "swim_counters_get": (C.c_int, [_H, C.POINTER(SwimCounters)]),
    "swim_last_error": (C.c_char_p, [_H]),
    "swim_is_overrides": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "swim_ceil_log2": (C.c_uint32, [C.c_uint32]),
}


# include/swimhip_shard.h (row-sharded multi-GPU handles; exported by libswimhip only, not by the oracle)
TRANSPORT_RCCL = 1
TRANSPORT_HOST = 2
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p, C.c_uint64,
                          C.POINTER(C.c_uint64))


class SwimShardSpec(C.Structure):
    _fields_ = [
        ("rank", C.c_uint32),
        ("world", C.c_uint32),
        ("transport", C.c_uint32),
        ("chunk_cap", C.c_uint32),
        ("rccl_id", C.c_uint8 * 128),
        ("exchange", EXCHANGE_FN),
        ("ctx", C.c_void_p),
        ("reserved", C.c_uint32 * 8),
    ]


SHARD_SIGNATURES = {
    "swim_rccl_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "swim_create_sharded": (C.c_int, [C.POINTER(SwimConfig), C.POINTER(SwimShardSpec), C.POINTER(_H)]),
    "swim_shard_range": (C.c_int, [_H, _U32P, _U32P]),
}


# include/swimhip_selftest.h (known-answer surface; exported by libswimhip and by the oracle)
SELFTEST_OVERRIDES, SELFTEST_PHILOX, SELFTEST_CLUSTER_MATH, SELFTEST_LOSS_ROLL = 0, 1, 2, 3
SELFTEST_SIGNATURES = {
    "swim_selftest_eval": (C.c_int, [C.c_uint32, _U32P, _U32P, C.c_size_t, C.c_uint32]),
}


def selftest_eval(lib, op, rows, device=0):
    """Evaluate `op` on a list of input tuples through swim_selftest_eval; returns a list of output tuples."""
    fn = lib.swim_selftest_eval
    fn.restype, fn.argtypes = SELFTEST_SIGNATURES["swim_selftest_eval"]
    win, wout = {SELFTEST_OVERRIDES: (4, 1), SELFTEST_PHILOX: (6, 4), SELFTEST_CLUSTER_MATH: (4, 4),
                 SELFTEST_LOSS_ROLL: (8, 1)}[op]
    flat = [int(x) & 0xFFFFFFFF for r in rows for x in r]
    assert len(flat) == win * len(rows)
    cin = (C.c_uint32 * max(1, len(flat)))(*flat)
    cout = (C.c_uint32 * max(1, wout * len(rows)))()
    rc = fn(op, cin, cout, len(rows), device)
    if rc != 0:
        raise RuntimeError(f"swim_selftest_eval(op={op}) rc={rc}")
    return [tuple(cout[i * wout:(i + 1) * wout]) for i in range(len(rows))]


# include/swimhip_debug.h (capacity-fallback counters; libswimhip only, with SWIM_CAPS / SWIM_FALLBACKS at create)
FB_NAMES = ["trk_walk", "ulog", "creq", "cwmax", "cev_slow", "replay", "mq", "sort_merge", "rx_all"]
DEBUG_SIGNATURES = {
    "swim_debug_fallbacks": (C.c_int, [_H, C.POINTER(C.c_uint64), C.c_size_t]),
    "swim_debug_caps": (C.c_int, [_H, C.POINTER(C.c_uint64), C.c_size_t]),
    "swim_debug_holders": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "swim_debug_set_incarnation": (C.c_int, [_H, C.c_uint32, C.c_uint32]),
}
CAP_NAMES = ["slots", "ring", "receipts", "replay", "history", "growths"]


def debug_caps(lib, handle):
    """{name: size} of the structures that grow between ticks (include/swimhip_debug.h swim_debug_caps)."""
    fn = lib.swim_debug_caps
    fn.restype, fn.argtypes = DEBUG_SIGNATURES["swim_debug_caps"]
    out = (C.c_uint64 * len(CAP_NAMES))()
    rc = fn(handle, out, len(CAP_NAMES))
    if rc != 0:
        raise RuntimeError(f"swim_debug_caps rc={rc}")
    return dict(zip(CAP_NAMES, (int(x) for x in out)))


def debug_holders(lib, handle, first, n):
    """[n][5] uint32 array: per member of [first, first + n) its gossip count, receipt-ring head and end positions,
    held-bit popcount and pending folded GOSSIP events (include/swimhip_debug.h swim_debug_holders)."""
    import numpy as np
    fn = lib.swim_debug_holders
    fn.restype, fn.argtypes = DEBUG_SIGNATURES["swim_debug_holders"]
    out = np.zeros((n, 5), dtype=np.uint32)
    rc = fn(handle, first, n, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    if rc != 0:
        raise RuntimeError(f"swim_debug_holders rc={rc}")
    return out


def debug_set_incarnation(lib, handle, m, inc):
    """Member m's own record at incarnation inc (include/swimhip_debug.h swim_debug_set_incarnation); the return code."""
    fn = lib.swim_debug_set_incarnation
    fn.restype, fn.argtypes = DEBUG_SIGNATURES["swim_debug_set_incarnation"]
    return fn(handle, m, inc)


def debug_fallbacks(lib, handle):
    """{name: count} of the capacity fallbacks the handle took (include/swimhip_debug.h)."""
    fn = lib.swim_debug_fallbacks
    fn.restype, fn.argtypes = DEBUG_SIGNATURES["swim_debug_fallbacks"]
    out = (C.c_uint64 * len(FB_NAMES))()
    rc = fn(handle, out, len(FB_NAMES))
    if rc != 0:
        raise RuntimeError(f"swim_debug_fallbacks rc={rc}")
    return dict(zip(FB_NAMES, (int(x) for x in out)))


# include/swimhip_wire.h (wire-format export; libswimhip only)
class SwimWireRecord(C.Structure):
    _fields_ = [("member", C.c_uint32), ("status", C.c_uint32), ("incarnation", C.c_uint32)]


WIRE_SYNC, WIRE_SYNC_ACK = 1, 2
_U8P = C.POINTER(C.c_uint8)
WIRE_SIGNATURES = {
    "swim_wire_sync_frame": (C.c_int, [C.c_uint32, C.c_uint32, C.c_char_p, C.c_char_p, C.POINTER(SwimWireRecord),
                                       C.c_size_t, _U8P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "swim_wire_gossip_frame": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(SwimWireRecord), _U8P,
                                         C.c_size_t, C.POINTER(C.c_size_t)]),
    "swim_export_sync_frame": (C.c_int, [_H, C.c_uint32, C.c_uint32, _U8P, C.c_size_t, C.POINTER(C.c_size_t)]),
}


def bind_wire(lib):
    for name, (res, args) in WIRE_SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def _frame_call(fn, *args):
    """Call an encoder twice: once for the size, once into a buffer of that size; returns the frame bytes."""
    n = C.c_size_t()
    fn(*args, None, 0, C.byref(n))
    buf = (C.c_uint8 * n.value)()
    rc = fn(*args, buf, n.value, C.byref(n))
    if rc != 0:
        raise RuntimeError(f"{fn.__name__} rc={rc}")
    return bytes(buf)


def wire_sync_frame(lib, kind, sender, records, cid=None, sync_group="default"):
    bind_wire(lib)
    arr = (SwimWireRecord * max(1, len(records)))(*[SwimWireRecord(*r) for r in records])
    return _frame_call(lib.swim_wire_sync_frame, kind, sender, cid.encode() if cid else None, sync_group.encode(),
                       arr, len(records))


def wire_gossip_frame(lib, sender, origin, counter, record):
    bind_wire(lib)
    return _frame_call(lib.swim_wire_gossip_frame, sender, origin, counter, C.byref(SwimWireRecord(*record)))


def export_sync_frame(lib, handle, observer, kind=WIRE_SYNC):
    bind_wire(lib)
    return _frame_call(lib.swim_export_sync_frame, handle, observer, kind)


def bind_shard(lib):
    """Attach the sharding entry points (engine library only)."""
    for name, (res, args) in SHARD_SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def bind(lib):
    """Attach restype/argtypes for every ABI symbol; raises AttributeError if one is missing."""
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def load(path):
    # RTLD_LOCAL keeps the oracle's and the engine's identically named swim_* symbols apart in one process
    return bind(C.CDLL(str(path), mode=C.RTLD_LOCAL))
