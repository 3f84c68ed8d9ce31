"""The CLI's first context, opened on a host thread while the interpreter imports the rest
(`python -m guacamole_amd`): HIP runtime and device initialisation (~0.15 s) is C code behind a
ctypes call that releases the GIL, so it overlaps numpy's and the commands' imports (~0.15 s)
instead of following them.  Nothing here imports numpy.  native.Context(device) adopts the
handle for its device once; any other context opens as usual.  Not used under a multi-process
launcher (WORLD_SIZE > 1): there torch must load its HIP runtime before libgqpileup.so
(distributed.check_hip_runtimes)."""
import ctypes
import os
import threading

_state = {}
_thread = None


def _open(path: str, device: int) -> None:
    try:
        lib = ctypes.CDLL(path)
        lib.gq_open.argtypes = [ctypes.c_int, ctypes.c_void_p]
        lib.gq_open.restype = ctypes.c_int
        h = ctypes.c_void_p()
        rc = lib.gq_open(int(device), ctypes.byref(h))
        _state["ctx"] = (int(device), rc, h)
    except Exception as e:  # (the ordinary open reports it)
        _state["err"] = e


def _map(path: str, lib_path: str) -> None:
    import time
    t0 = time.perf_counter()
    try:
        lib = ctypes.CDLL(lib_path)
        lib.gq_bam_dev_map_ex.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_void_p]
        lib.gq_bam_dev_map_ex.restype = ctypes.c_int
        h = ctypes.c_void_p()
        rc = lib.gq_bam_dev_map_ex(path.encode(), 1, ctypes.byref(h))
        _maps[path] = (rc, h, t0, time.perf_counter())
    except Exception:
        pass


_maps = {}
_map_threads = {}


def take_map(path: str):
    """The early host map of `path` (gq_bam_dev_map_ex, populated): (rc, handle, t_start,
    t_mapped) once, or None."""
    th = _map_threads.pop(path, None)
    if th is None:
        return None
    th.join()
    return _maps.pop(path, None)


def start(argv) -> None:
    """Open the context of the command's --device (default 0) on a host thread, and map the
    command's BAM inputs (--reads, --tumor-reads, --normal-reads) on others."""
    global _thread
    if int(os.environ.get("WORLD_SIZE", "1") or 1) > 1 or os.environ.get("GQ_EARLY_OPEN", "1") == "0":
        return
    device = 0
    for i, a in enumerate(argv):
        if a == "--device" and i + 1 < len(argv):
            try:
                device = int(argv[i + 1])
            except ValueError:
                return
        elif a.startswith("--device="):
            try:
                device = int(a.split("=", 1)[1])
            except ValueError:
                return
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.environ.get("GQ_LIB", os.path.join(here, "_lib", "libgqpileup.so"))
    if not os.path.exists(path):
        return
    _thread = threading.Thread(target=_open, args=(path, device), name="gq_early_open", daemon=True)
    _thread.start()
    if os.environ.get("GQ_INGEST", "device") == "host":
        return
    for i, a in enumerate(argv[:-1]):
        b = argv[i + 1]
        if a in ("--reads", "--tumor-reads", "--normal-reads") and b.lower().endswith(".bam") and os.path.isfile(b):
            if b not in _map_threads:
                _map_threads[b] = threading.Thread(target=_map, args=(b, path), name="gq_early_map", daemon=True)
                _map_threads[b].start()


def take(device: int):
    """The early context's handle for `device` (once), or None."""
    global _thread
    if _thread is None:
        return None
    _thread.join()
    _thread = None
    got = _state.pop("ctx", None)
    if got is None or got[0] != int(device) or got[1] != 0:
        return None
    return got[2]
