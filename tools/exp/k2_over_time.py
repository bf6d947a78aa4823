"""K2 (q + codes) on ONE fixed set of buffers, timed 30 times over ~10 s, with the GPU's current
memory / system clock levels read from sysfs when readable.  If the 1.7 / 2.0 ms modes appear
with fixed buffers, the slow mode is a time-dependent GPU state, not placement.
    python tools/exp/k2_over_time.py"""
import ctypes, glob, json, os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _card():
    """sysfs card of the active device: the one whose PCI bus id matches torch's device."""
    try:
        bus = torch.cuda.get_device_properties(torch.cuda.current_device()).pci_bus_id
    except Exception:
        bus = None
    for p in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            if bus is not None and os.path.basename(os.path.realpath(p)).endswith(f"{bus:02x}:00.0"):
                return p
        except OSError:
            pass
    return None


def clocks(card):
    """Current memory / system clock levels of the active device's card, as the flat keys of
    profiles/r01g_exp_k2_over_time.jsonl (mclk0 / sclk0 = the line marked current).  That
    file came from an earlier revision which always read card0; this one reads the card of
    the device under test (empty when sysfs is not readable)."""
    out = {}
    if card is None:
        return out
    for key, f in (("mclk0", "pp_dpm_mclk"), ("sclk0", "pp_dpm_sclk")):
        try:
            cur = [l.strip() for l in open(os.path.join(card, f)) if l.strip().endswith("*")]
            out[key] = cur[0] if cur else "?"
        except OSError:
            pass
    return out


def main():
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    n, d = 1024, 1 << 20
    m = uqdme.rate_to_m(1, d)
    x = torch.randn(n, d, device="cuda")
    q = torch.empty_like(x)
    c = torch.empty((n, d), dtype=torch.int8, device="cuda")
    X = torch.rand(n, device="cuda")
    l1 = torch.empty(n, device="cuda")
    b = ctypes.c_size_t()
    lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
    ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
    ovf = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")
    f = lambda: lib.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), c.data_ptr(), ovf.data_ptr(), n, d, m,
                                               X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
    card = _card()
    t0 = time.time()
    for trial in range(30):
        for _ in range(2):
            _lib.check(f(), "k2")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"trial": trial, "t_s": round(time.time() - t0, 2), "k2_ms": round(e0.elapsed_time(e1) / 5, 4),
                          **clocks(card)}), flush=True)
        time.sleep(0.25)


if __name__ == "__main__":
    main()
