"""Full-frame pins (tests/golden/frame_<cfg>.npz, written by tests/golden/make_frames.py)
and the checks that compare a rendered frame with them.

A frame is summarised without storing it (7.4 MB of incompressible floats per frame):
  <p>_sha256          sha256 of the H*W*3 float32 frame, NaN bit patterns canonicalised
                      (the whole-frame bit-exact pin);
  <p>_rowxor/_colxor  per row / column and channel XOR of the float bit patterns (they
                      locate any differing pixel);
  <p>_blocks          8x8 block means; <p>_crops 64x64 full-resolution crops;
  <p>_nonfinite       flat indices of pixels with a non-finite component.
"""
import hashlib

import numpy as np

CROP = 64


def canon_bits(img):
    """float32 bit patterns with every NaN as 0x7fc00000 (CPU and GPU NaN payloads differ)."""
    a = np.array(img, np.float32, copy=True)
    bits = a.view(np.uint32)
    bits[np.isnan(a)] = 0x7FC00000
    return bits


def block_means(img, b=8):
    h, w = img.shape[:2]
    return img.reshape(h // b, b, w // b, b, 3).astype(np.float64).mean((1, 3)).astype(np.float32)


def crops(img, origins):
    return np.stack([img[r:r + CROP, c:c + CROP] for r, c in origins])


def frame_blocks(img, prefix, origins):
    return {prefix + "_blocks": block_means(img), prefix + "_crops": crops(img, origins)}


def frame_summary(img, prefix, origins):
    bits = canon_bits(img)
    out = {prefix + "_sha256": np.array(hashlib.sha256(bits.tobytes()).hexdigest()),
           prefix + "_rowxor": np.bitwise_xor.reduce(bits, axis=1).astype(np.uint32),
           prefix + "_colxor": np.bitwise_xor.reduce(bits, axis=0).astype(np.uint32)}
    out.update(frame_blocks(img, prefix, origins))
    h, w = img.shape[:2]
    out[prefix + "_nonfinite"] = np.nonzero(~np.isfinite(img.reshape(-1, 3)).all(1))[0].astype(np.int64)
    return out


def rel_l2_rows(a, b):
    a = np.asarray(a, np.float64).reshape(-1, 3)
    b = np.asarray(b, np.float64).reshape(-1, 3)
    num = np.linalg.norm(a - b, axis=1)
    den = np.maximum(np.linalg.norm(b, axis=1), 1e-12)
    r = num / den
    r[num == 0] = 0.0
    return r


def check_exact(img, g, prefix, what):
    """img bit-for-bit equal to the pinned frame: sha256, and on a mismatch the
    differing rows / columns (from the XOR pins) in the assertion message."""
    bits = canon_bits(img)
    sha = hashlib.sha256(bits.tobytes()).hexdigest()
    if sha != str(g[prefix + "_sha256"]):
        rows = np.nonzero((np.bitwise_xor.reduce(bits, axis=1) != g[prefix + "_rowxor"]).any(1))[0]
        cols = np.nonzero((np.bitwise_xor.reduce(bits, axis=0) != g[prefix + "_colxor"]).any(1))[0]
        raise AssertionError("%s: frame differs from the reference's; rows %s cols %s" % (what, rows[:20], cols[:20]))
    nf = np.nonzero(~np.isfinite(img.reshape(-1, 3)).all(1))[0]
    assert np.array_equal(nf, g[prefix + "_nonfinite"]), (what, nf, g[prefix + "_nonfinite"])
    # redundant with the hash, but states the pins a reader can check by eye
    assert np.array_equal(canon_bits(crops(img, g["crop_origins"])), canon_bits(g[prefix + "_crops"]))
    return True


def check_close(img, g, prefix, what, tol_blocks, tol_crop_q99, tol_crop_max):
    """Frames that are sums of fp32 atomics (BDPT splats): 8x8 block means within
    relative L2 tol_blocks, crop pixels within the given quantile / max.  Non-finite
    values must sit where the reference's are: the blocks (and crop pixels) that are
    non-finite in the pin and in img must be the same ones, and the finiteness mask of
    the comparison comes from the pin alone, so a GPU NaN / Inf is a failure, never a
    dropped block."""
    gb, ib = g[prefix + "_blocks"], block_means(img)
    fin = np.isfinite(gb).all(-1)
    bad = np.nonzero(fin != np.isfinite(ib).all(-1))
    assert bad[0].size == 0, (what, "non-finite 8x8 blocks differ from the reference's at", list(zip(*bad))[:10])
    r = rel_l2_rows(ib[fin], gb[fin])
    gc, ic = g[prefix + "_crops"], crops(img, g["crop_origins"])
    cfin = np.isfinite(gc).all(-1)
    assert np.array_equal(cfin, np.isfinite(ic).all(-1)), (what, "non-finite crop pixels differ from the reference's")
    c = rel_l2_rows(ic[cfin], gc[cfin])
    print("%s: block relL2 max %.3g, crop relL2 q99 %.3g max %.3g" % (what, r.max(), np.quantile(c, 0.99), c.max()))
    assert r.max() <= tol_blocks, (what, r.max())
    assert np.quantile(c, 0.99) <= tol_crop_q99 and c.max() <= tol_crop_max, (what, np.quantile(c, 0.99), c.max())
