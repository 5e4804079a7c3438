"""Host-buffer collide pipeline (VERDICT r5 "next" #1).

CPU: mplib_amd/csrc/mpg_hostpipe.h -- the chunk plan, the slot protocol
between the input feeder thread and the issuing thread, and the unpacking of
the packed mask rows -- driven by tests/native/hostpipe_test.cpp with a fake
device (random delays, slot inputs read late so an early refill shows up),
ragged sizes at the chunk boundaries, one to three slots, injected failures;
built once plain and once under ThreadSanitizer when the compiler has it.

GPU: the real pipeline (mpg_collide_batch with MPG_MEM_HOST above the latency
path's sizes) against the oracle at ragged sizes and small chunks
(MPG_HOST_CHUNK), flags only, and link-pose input."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "hostpipe_test.cpp")


def _build_run(extra):
    out = os.path.join(tempfile.gettempdir(), "mplib_amd_hostpipe_%d_%d%s" % (os.getuid(), os.getpid(),
                                                                               "_tsan" if extra else ""))
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", *extra, "-o", out, SRC])
    r = subprocess.run([out], capture_output=True, text=True, timeout=300)
    os.unlink(out)
    return r


def test_pipeline_protocol_fake_device():
    r = _build_run([])
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr


def test_pipeline_protocol_thread_sanitizer():
    probe = subprocess.run(["g++", "-fsanitize=thread", "-x", "c++", "-", "-o", os.devnull],
                           input="int main(){}", capture_output=True, text=True)
    if probe.returncode != 0:
        pytest.skip("g++ without ThreadSanitizer")
    r = _build_run(["-g", "-fsanitize=thread"])
    assert r.returncode == 0 and r.stdout.startswith("ok") and "WARNING: ThreadSanitizer" not in r.stderr, \
        r.stdout + r.stderr[-4000:]


# ------------------------------------------------------------------ GPU
_OW = {}


def _ow(cfg):
    import worlds as Wd
    if cfg not in _OW:
        _OW[cfg] = Wd.oracle_world(cfg)
    return _OW[cfg]


def _small_chunk_world(monkeypatch, cfg, chunk):
    import worlds as Wd
    from mplib_amd.batch import DeviceWorld
    monkeypatch.setenv("MPG_HOST_CHUNK", str(chunk))
    return DeviceWorld(Wd.desc_arrays(_ow(cfg)))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1025, 4095, 4097, 12289, 70001])
def test_host_pipeline_ragged_chunks_match_oracle(monkeypatch, n):
    """Chunks of 4096 configurations (MPG_HOST_CHUNK): ragged last chunks,
    every slot of the ring reused many times, flags and pair bits vs the
    oracle."""
    import worlds as Wd
    d = _small_chunk_world(monkeypatch, 3, 4096)
    q = Wd.sample_q(_ow(3).art, n, 9100 + n)
    f, m = d.collide_batch(q)
    fo, mo = _ow(3).collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(f, fo)
    np.testing.assert_array_equal(m, mo)
    d.close()


@pytest.mark.gpu
def test_host_pipeline_flags_only_and_repeat(monkeypatch):
    """pair_mask = NULL (flags only), and the same world called again with a
    different size (the ring's buffers are reused, nothing stale leaks)."""
    import ctypes
    import worlds as Wd
    from mplib_amd import _capi as C
    d = _small_chunk_world(monkeypatch, 3, 2048)
    for n, seed in ((9000, 1), (3000, 2), (20000, 3)):
        q = Wd.sample_q(_ow(3).art, n, 9300 + seed)
        fl = np.full(n, 0xAB, np.uint8)
        C.check(C.lib().mpg_collide_batch(d.handle, q.ctypes.data_as(ctypes.c_void_p), n,
                                          fl.ctypes.data_as(ctypes.c_void_p), None, C.MPG_MEM_HOST, None),
                "mpg_collide_batch")
        fo, _ = _ow(3).collide_batch(q, nthreads=min(16, os.cpu_count() or 1))
        np.testing.assert_array_equal(fl, fo)
        f, m = d.collide_batch(q)
        np.testing.assert_array_equal(f, fo)
    d.close()


@pytest.mark.gpu
def test_host_pipeline_link_pose_input(monkeypatch):
    """mpg_collide_link_poses with host buffers through the pipeline (rows of
    n_links * 7 doubles): the same bits as the joint-state input."""
    import ctypes
    import worlds as Wd
    from mplib_amd import _capi as C
    d = _small_chunk_world(monkeypatch, 3, 1024)
    n = 6000
    q = Wd.sample_q(_ow(3).art, n, 9400)
    poses = np.ascontiguousarray(d.fk_batch(q))
    fl = np.zeros(n, np.uint8)
    pm = np.zeros((n, d.mask_words), np.uint32)
    C.check(C.lib().mpg_collide_link_poses(d.handle, poses.ctypes.data_as(ctypes.c_void_p), n,
                                           fl.ctypes.data_as(ctypes.c_void_p), pm.ctypes.data_as(ctypes.c_void_p),
                                           C.MPG_MEM_HOST, None), "mpg_collide_link_poses")
    f, m = d.collide_batch(q)
    np.testing.assert_array_equal(fl, f)
    np.testing.assert_array_equal(pm, m)
    d.close()
