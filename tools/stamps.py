"""Phase breakdown of the encode kernel from a -DFG_STAMPS build (diagnostic only)."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-flac_amd"))
import numpy as np, torch
import flacgpu, synth

NAMES = ["DMA issue+job load", "sample load", "waste+eq", "bestOrder", "rice pass", "param search (rest)",
         "desc+rec+bar", "stereo+exact", "ticket atomic", "vmcnt(0) wait", "top barrier",
         "fixed rice search", "LPC load+autocorr", "LPC Levinson-Durbin", "LPC residual pass",
         "bestOrder before i64"]
PNAMES = ["top barrier", "offsets+bar", "zero img+bars", "residuals", "pack codes+bar", "CRC+bars", "store+bar",
          "ticket+desc loads", "vmcnt(0) wait", "DMA issue+sample load", "lane_bits/bits loads+scan"]
S, F = int(os.environ.get("STAMP_S", "1024")), int(os.environ.get("STAMP_F", "32"))
CH, BITS, RATE = int(os.environ.get("CH", "2")), int(os.environ.get("BITS", "16")), int(os.environ.get("RATE", "44100"))
FB = CH * BITS // 8
LPC = int(os.environ.get("LPC", "0"))
enc = flacgpu.Encoder(CH, BITS, RATE, max_frames=S * F, lpc_order=LPC)
L = enc.lib
L.flacgpu_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
pool = synth.synth_samples(4096 * 256, CH, BITS, RATE)
pcm = np.frombuffer(synth.to_pcm_bytes(pool, BITS), dtype=np.uint8)
buf = np.concatenate([pcm[(s % 8) * 4096 * FB * 16:][: F * 4096 * FB] for s in range(S)])
plan = enc.plan([s * F * 4096 * FB for s in range(S)], [F * 4096] * S)
d_pcm = torch.from_numpy(buf).cuda()
d_out = torch.empty(int(plan.out_bound), dtype=torch.uint8, device="cuda")
d_fb = torch.empty(plan.n_frames, dtype=torch.int32, device="cuda")
d_off = torch.empty(plan.n_frames, dtype=torch.int64, device="cuda")
d_tot = torch.zeros(2, dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
run = lambda: enc.encode_plan_device(plan, d_pcm.data_ptr(), d_out.data_ptr(), int(plan.out_bound), d_fb.data_ptr(),
                                     d_off.data_ptr(), d_tot.data_ptr(), None, st.cuda_stream)
run(); torch.cuda.synchronize()
out = (ctypes.c_uint64 * 32)()
print("stamps supported:", L.flacgpu_debug_stamps(enc.ctx, out, 1) == 0)
enc.set_timing(True)
for _ in range(5):
    run()
torch.cuda.synchronize()
print("encode ms/launch", enc.kernel_time(0))
L.flacgpu_debug_stamps(enc.ctx, out, 0)
WA = 4 if CH == 2 else CH                        # analysis waves per frame (stereo: L, R, M, S)
NOUT = 2 if CH == 2 else CH
if CH == 2 and BITS == 16 and LPC == 0:
    WP = 8                                         # k_pack4: 4 waves per written subframe
elif BITS == 32 or NOUT > 2:
    WP = NOUT * (4 if NOUT <= 4 else 2)            # k_packw: WPS waves per written subframe
else:
    WP = NOUT                                      # k_pack: one wave per written subframe
for base, names, label in [(0, NAMES, "analysis"), (16, PNAMES, "pack")]:
    tot = sum(out[base:base + len(names)])
    print(f"-- {label}")
    for i, n in enumerate(names):
        v = out[base + i]
        print(f"{i:2d} {n:20s} {v / max(tot,1) * 100:6.2f}%  {v / (5 * S * F * (WA if base == 0 else WP)):10.1f} clk/wave-frame")
