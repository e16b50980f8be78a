"""Generate the golden fixtures under tests/golden/ from the CPU restatement
(oracle/neo_oracle.c) and check every one against float64 numpy truth.

Inputs: splitmix64 -> U[-1,1) float32 (oracle.noise), seeds in the file names.
The reference itself cannot be built here ("Oracle"), so the
fixtures pin our GPU path to the restatement, and the restatement to float64
truth (max errors recorded in manifest.json) and to the reference's own KATs
(tests/test_oracle.py).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402


def peak(y, ref):
    return float(np.abs(np.asarray(y, np.complex128) - ref).max() / np.abs(ref).max())


def main():
    manifest = {}

    # (1) C1: 1024-pt c2c forward + backward, seed 1
    x = O.noise(1, 2048).view(np.complex64)
    X = O.fft(x)
    xb = O.ifft(X)
    manifest["c2c_1024_seed1"] = {"fwd_vs_f64": peak(X, np.fft.fft(x.astype(np.complex128))),
                                  "bwd_vs_f64": peak(xb, 1024 * np.fft.ifft(X.astype(np.complex128)))}
    np.savez(os.path.join(HERE, "c2c_1024_seed1.npz"), x=x, fwd=X, bwd=xb)

    # (2) 4096 x 8 batches forward, seed 2 (C2 transform size)
    x = O.noise(2, 2 * 4096 * 8).view(np.complex64).reshape(8, 4096)
    X = O.fft(x)
    manifest["c2c_4096x8_seed2"] = {"fwd_vs_f64": peak(X, np.fft.fft(x.astype(np.complex128), axis=-1))}
    np.savez(os.path.join(HERE, "c2c_4096x8_seed2.npz"), x=x, fwd=X)

    # (3) rfft / irfft 512 and 1024, seed 3
    for n in (512, 1024):
        r = O.noise(3, n)
        R = O.rfft(r)
        back = O.irfft(R, n)
        manifest[f"rfft_{n}_seed3"] = {"r2c_vs_f64": peak(R, np.fft.rfft(r.astype(np.float64))),
                                       "c2r_vs_f64": peak(back, n * r.astype(np.float64))}
        np.savez(os.path.join(HERE, f"rfft_{n}_seed3.npz"), x=r, r2c=R, c2r=back)

    # (4) uniform_partition: 3000-tap IR at B=256 -> [1,12,257]; 2-ch normalized IR at B=128
    ir = O.noise(4, 3000)
    H = O.uniform_partition(ir[None], 256)
    truth = np.stack([np.fft.rfft(np.pad(ir[p * 256:(p + 1) * 256].astype(np.float64), (0, 512 - len(ir[p * 256:(p + 1) * 256]))))
                      for p in range(12)])
    manifest["partition_3000_b256_seed4"] = {"vs_f64": peak(H[0], truth), "shape": list(H.shape)}
    ir2 = np.stack([O.noise(40, 1500), O.noise(41, 1500) * 0.5]).astype(np.float32)
    irn = O.normalize_impulse(ir2)
    H2 = O.uniform_partition(irn, 128)
    np.savez(os.path.join(HERE, "partition_seed4.npz"), ir=ir, H=H, ir2=ir2, ir2_norm=irn, H2=H2)

    # (5) UPOLS outputs
    cases = [("upols_b512_l4096_seed5", 512, 4096, 1, 40, 5),
             ("upols_b256_l2560_2ch_seed6", 256, 2560, 2, 40, 6),
             ("upols_b512_l96000_seed7", 512, 96000, 1, 200, 7)]
    for name, B, L, C, nb, seed in cases:
        ir = np.stack([O.noise(seed * 100 + c, L) for c in range(C)])
        irn = O.normalize_impulse(ir)
        parts = O.uniform_partition(irn, B)
        sig = np.stack([O.noise(seed * 1000 + c, B * nb) for c in range(C)])
        out = O.dense_convolve(sig, parts)
        errs = []
        for c in range(C):
            truth = np.convolve(sig[c].astype(np.float64), irn[c].astype(np.float64))[: B * nb]
            errs.append(peak(out[c], truth))
        manifest[name] = {"B": B, "L": L, "C": C, "blocks": nb, "vs_f64_direct": max(errs),
                          "P": int(parts.shape[1])}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), ir=ir, signal=sig, out=out)

    # (5b) UPOLA (upola_convolver) output, 2 ch, B=256, L=2560, 40 blocks
    B, L, C, nb, seed = 256, 2560, 2, 40, 8
    ir = np.stack([O.noise(seed * 100 + c, L) for c in range(C)])
    irn = O.normalize_impulse(ir)
    parts = O.uniform_partition(irn, B)
    sig = np.stack([O.noise(seed * 1000 + c, B * nb) for c in range(C)])
    out = O.dense_convolve(sig, parts, method="upola")
    errs = [peak(out[c], np.convolve(sig[c].astype(np.float64), irn[c].astype(np.float64))[: B * nb]) for c in range(C)]
    manifest["upola_b256_l2560_2ch_seed8"] = {"B": B, "L": L, "C": C, "blocks": nb, "vs_f64_direct": max(errs)}
    np.savez_compressed(os.path.join(HERE, "upola_b256_l2560_2ch_seed8.npz"), ir=ir, signal=sig, out=out)

    # (5c) fft_convolve / direct_convolve, signal 5000, patch 777, seed 9
    x, p = O.noise(90, 5000), O.noise(91, 777)
    fc, dc = O.fft_convolve(x, p), O.direct_convolve(x, p)
    t = np.convolve(x.astype(np.float64), p.astype(np.float64))
    manifest["convolve_5000x777_seed9"] = {"fft_vs_f64": peak(fc, t), "direct_vs_f64": peak(dc, t)}
    np.savez(os.path.join(HERE, "convolve_5000x777_seed9.npz"), signal=x, patch=p, fft=fc, direct=dc)

    # (6) multiply_add KAT (multiply_add_test.cpp:52-95)
    for n in (2, 33, 128):
        y = O.multiply_add(np.full(n, 1 + 2j, np.complex64), np.full(n, 3 + 4j, np.complex64),
                           np.full(n, 5 + 6j, np.complex64))
        assert np.all(y == 0 + 16j)
    manifest["multiply_add_kat"] = {"ok": True}

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
