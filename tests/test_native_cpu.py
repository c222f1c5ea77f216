"""CPU checks of ABI 4 (no device calls): the shard arithmetic of batches and
multi-device engines (contiguous [g n / G, (g + 1) n / G)),
the cls_config layout, and that the batch / multi-device / RCCL entry
points refuse null handles with CLS_E_INVAL instead of touching a device."""
import ctypes as C

import pytest

from vpp_amd import _abi
from vpp_amd.engine import shard_range

SIZES = [0, 1, 3, 7, 8, 9, 255, 1000, (1 << 20) + 13, 1 << 28, (1 << 31) + 5, 2 << 30, (1 << 40) + 3,
         (1 << 62) + 11]


@pytest.mark.parametrize("G", [1, 2, 3, 4, 5, 7, 8])
def test_shards_cover_contiguously_and_balance(G):
    for n in SIZES:
        parts = [shard_range(n, G, g) for g in range(G)]
        assert parts[0][0] == 0
        for (a, k), (b, _) in zip(parts, parts[1:]):
            assert a + k == b                       # contiguous
        assert parts[-1][0] + parts[-1][1] == n     # covers [0, n)
        counts = [k for _, k in parts]
        assert max(counts) - min(counts) <= 1       # balanced
        assert [a for a, _ in parts] == [g * n // G for g in range(G)]


def test_config4_split_over_eight():
    # 2 Gi packets over 8 GPUs: 256 Mi each, the config-3 batch per GPU
    assert [shard_range(2 << 30, 8, g) for g in range(8)] == [(g << 28, 1 << 28) for g in range(8)]


def test_shard_range_refuses_bad_arguments():
    L = _abi.lib()
    a, b = C.c_uint64(), C.c_uint64()
    assert L.cls_shard_range(10, 0, 0, C.byref(a), C.byref(b)) == _abi.E_INVAL
    assert L.cls_shard_range(10, 4, 4, C.byref(a), C.byref(b)) == _abi.E_INVAL
    assert L.cls_shard_range(10, 4, 0, None, C.byref(b)) == _abi.E_INVAL


def test_config_layout_keeps_abi3_size():
    # ABI 3's cls_config was {int device; uint32 reserved[7]}: 32 bytes
    assert C.sizeof(_abi.Config) == 32
    assert _abi.Config.devices.offset == 8


def test_null_handles_are_refused():
    L = _abi.lib()
    p = C.c_void_p()
    u = C.c_uint32()
    assert L.cls_batch_create(None, _abi.AF_V4, 16, 0, C.byref(p)) == _abi.E_INVAL
    assert L.cls_classify_batch(None, 1, None, None, 0) == _abi.E_INVAL
    assert L.cls_batch_connect(None, None, 0) == _abi.E_INVAL
    assert L.cls_batch_wait(None) == _abi.E_INVAL
    assert L.cls_batch_upload(None, 0, 0, 1, None) == _abi.E_INVAL
    assert L.cls_batch_download(None, 0, 0, 1, None) == _abi.E_INVAL
    assert L.cls_batch_counters(None, None, 0) == _abi.E_INVAL
    assert L.cls_batch_shards(None, C.byref(u)) == _abi.E_INVAL
    assert L.cls_engine_devices(None, C.byref(u)) == _abi.E_INVAL
    assert L.cls_device_engine(None, 0, C.byref(p)) == _abi.E_INVAL
    assert L.cls_comm_init(None, 1, 0, None) == _abi.E_INVAL
    assert L.cls_comm_info(None, None, None) == _abi.E_INVAL
    assert L.cls_comm_unique_id(None) == _abi.E_INVAL
    L.cls_batch_destroy(None)                       # a no-op


def test_multi_device_engine_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    from vpp_amd.engine import Engine
    with pytest.raises(_abi.ClsError):
        Engine(devices=[0, 1])
