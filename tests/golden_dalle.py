"""Golden re-statement of the dalle-pytorch sparse attention layers, written the way the pinned fork
computes them (pad the sequence by one token, split text / image, einsum over an axial reshape or
an unfold window, joint softmax over [text keys || local keys]). Used only by tests to pin the
semantics of ``dalle_amd.models.patterns`` (the static-mask form every kernel implements)."""
import torch
import torch.nn.functional as F


def _neg(t):
    return -torch.finfo(t.dtype).max


def text_attention(q_text, k_text, v_text):
    dots = torch.einsum("bid,bjd->bij", q_text, k_text)
    i, j = dots.shape[-2:]
    mask = torch.ones(i, j, dtype=torch.bool).triu_(j - i + 1)
    dots = dots.masked_fill(mask, _neg(dots))
    return torch.einsum("bij,bjd->bid", dots.softmax(-1), v_text)


def axial_attention(q, k, v, text_len, img_size, axis):
    """q, k, v: (bh, n+1 padded, d) already rotated & q scaled."""
    img_seq_len = img_size * img_size
    qt, qi = q[:, :-img_seq_len], q[:, -img_seq_len:]
    kt, ki = k[:, :-img_seq_len], k[:, -img_seq_len:]
    vt, vi = v[:, :-img_seq_len], v[:, -img_seq_len:]
    out_text = text_attention(qt, kt, vt)

    def split(t):
        t = t.reshape(t.shape[0], img_size, img_size, t.shape[-1])
        return t if axis == 0 else t.transpose(1, 2)

    qi, ki, vi = split(qi), split(ki), split(vi)
    dots_ii = torch.einsum("bxid,bxjd->bxij", qi, ki)
    dots_it = torch.einsum("bxid,bjd->bxij", qi, kt)
    dots = torch.cat([dots_it, dots_ii], dim=-1)
    i = img_size
    causal = torch.ones(i, img_size, dtype=torch.bool).triu_(img_size - i + 1)
    mask = torch.cat([torch.zeros(i, text_len, dtype=torch.bool), causal], dim=-1)
    dots = dots.masked_fill(mask, _neg(dots))
    attn = dots.softmax(-1)
    a_t, a_i = attn[..., :text_len], attn[..., text_len:]
    out_img = torch.einsum("bxij,bxjd->bxid", a_i, vi) + torch.einsum("bxij,bjd->bxid", a_t, vt)
    if axis == 1:
        out_img = out_img.transpose(1, 2)
    out_img = out_img.reshape(out_img.shape[0], img_seq_len, -1)
    return torch.cat([out_text, out_img], dim=1)


def conv_attention(q, k, v, text_len, img_size, kernel_size=5):
    """Upper-left k x k causal window (causal padding (k-1, 0, k-1, 0)), joint softmax with text."""
    img_seq_len = img_size * img_size
    qt, qi = q[:, :-img_seq_len], q[:, -img_seq_len:]
    kt, ki = k[:, :-img_seq_len], k[:, -img_seq_len:]
    vt, vi = v[:, :-img_seq_len], v[:, -img_seq_len:]
    out_text = text_attention(qt, kt, vt)
    pad = kernel_size - 1

    def unfold(t):
        t = t.reshape(t.shape[0], img_size, img_size, -1).permute(0, 3, 1, 2)
        t = F.pad(t, (pad, 0, pad, 0))
        t = F.unfold(t, kernel_size)  # (b, d*k*k, i)
        return t.reshape(t.shape[0], -1, kernel_size * kernel_size, img_seq_len).permute(0, 3, 2, 1)  # (b, i, j, d)

    ku, vu = unfold(ki), unfold(vi)
    dots_img = torch.einsum("bid,bijd->bij", qi, ku)
    dots_text = torch.einsum("bid,bjd->bij", qi, kt)
    idx = torch.arange(img_seq_len, dtype=torch.float32).reshape(1, 1, img_size, img_size)
    idx = F.pad(idx, (pad, 0, pad, 0), value=float(img_seq_len))
    idx = F.unfold(idx, kernel_size).transpose(1, 2)  # (1, i, j)
    causal = torch.arange(img_seq_len).reshape(1, -1, 1) < idx
    dots = torch.cat([dots_text, dots_img], dim=-1)
    mask = torch.cat([torch.zeros(1, img_seq_len, text_len, dtype=torch.bool), causal], dim=-1)
    dots = dots.masked_fill(mask, _neg(dots))
    attn = dots.softmax(-1)
    a_t, a_i = attn[..., :text_len], attn[..., text_len:]
    out_img = torch.einsum("bij,bijd->bid", a_i, vu) + torch.einsum("bij,bjd->bid", a_t, vt)
    return torch.cat([out_text, out_img], dim=1)
