"""TF-convention padding arithmetic (NHWC)."""


def _pair(v):
    if isinstance(v, (list, tuple)):
        if len(v) == 4:      # TF [1, h, w, 1]
            return int(v[1]), int(v[2])
        if len(v) == 2:
            return int(v[0]), int(v[1])
        if len(v) == 1:
            return int(v[0]), int(v[0])
    return int(v), int(v)


def same_pads(in_size, k, s, d=1):
    """(pad_before, pad_after, out) for TF 'SAME' along one axis."""
    k_eff = (k - 1) * d + 1
    out = -(-in_size // s)
    total = max((out - 1) * s + k_eff - in_size, 0)
    return total // 2, total - total // 2, out


def conv_geometry(h, w, kh, kw, strides, padding, dilations=1):
    """Return (out_h, out_w, pad_t, pad_b, pad_l, pad_r)."""
    sh, sw = _pair(strides)
    dh, dw = _pair(dilations)
    if isinstance(padding, str):
        p = padding.upper()
        if p == "SAME":
            pt, pb, oh = same_pads(h, kh, sh, dh)
            pl, pr, ow = same_pads(w, kw, sw, dw)
            return oh, ow, pt, pb, pl, pr
        if p == "VALID":
            oh = (h - ((kh - 1) * dh + 1)) // sh + 1
            ow = (w - ((kw - 1) * dw + 1)) // sw + 1
            return oh, ow, 0, 0, 0, 0
        raise ValueError("padding must be SAME or VALID, got %r" % padding)
    if isinstance(padding, int):
        pt = pb = pl = pr = padding
    elif len(padding) == 2:
        pt = pb = int(padding[0])
        pl = pr = int(padding[1])
    else:
        pt, pb, pl, pr = (int(x) for x in padding)
    oh = (h + pt + pb - ((kh - 1) * dh + 1)) // sh + 1
    ow = (w + pl + pr - ((kw - 1) * dw + 1)) // sw + 1
    return oh, ow, pt, pb, pl, pr


pair = _pair
