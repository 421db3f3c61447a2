"""K20: the VQGAN decoder on the hand-written HIP kernels (implicit-GEMM MFMA 3x3 convs with fused
GroupNorm+SiLU input, folded 2x upsampling, fused residual; attention block; fused RGB output conv)
vs the fp32 PyTorch taming decoder."""
import pytest
import torch

from dalle_amd.models.vqgan import VQGanVAE

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_conv3x3_kernel_vs_torch(cuda):
    C = __import__("dalle_amd.ops.ext", fromlist=["x"]).load_extension(required=True)
    torch.manual_seed(0)
    for (n, h, w, cin, cout, ups, gn) in [(2, 16, 16, 128, 256, False, True), (1, 8, 16, 256, 128, True, False),
                                           (2, 32, 32, 64, 128, False, True)]:
        x = torch.randn(n, h, w, cin, device=cuda)
        conv = torch.nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
        norm = torch.nn.GroupNorm(32, cin, eps=1e-6).to(cuda)
        with torch.no_grad():
            norm.weight.uniform_(0.5, 1.5)
            norm.bias.uniform_(-0.3, 0.3)
        xin = x.permute(0, 3, 1, 2)
        if gn:
            xin = torch.nn.functional.silu(norm(xin))
        if ups:
            xin = torch.nn.functional.interpolate(xin, scale_factor=2.0, mode="nearest")
        res = torch.randn(n, xin.shape[2], xin.shape[3], cout, device=cuda).bfloat16()
        ref = conv(xin).permute(0, 2, 3, 1) + res.float()
        wk = conv.weight.detach().permute(0, 2, 3, 1).reshape(cout, -1).bfloat16().contiguous()
        xb = x.bfloat16().contiguous()
        if gn:
            mean, rstd = C.gn_stats(xb, 1e-6)
            ref_m = xb.float().view(n, -1, 32, cin // 32).mean(dim=(1, 3))
            assert torch.allclose(mean, ref_m, atol=1e-4)
            y = C.conv3x3(xb, wk, conv.bias.detach().float(), res, mean, rstd, norm.weight.detach().float(),
                          norm.bias.detach().float(), ups=ups)
        else:
            y = C.conv3x3(xb, wk, conv.bias.detach().float(), res, ups=ups)
        assert y.shape == ref.shape
        assert _rel(y, ref) < 2e-2, (n, h, w, cin, cout, ups, gn, _rel(y, ref))


@pytest.mark.parametrize("n,h,w,cin", [(2, 256, 256, 128), (1, 40, 24, 64), (2, 16, 48, 32)])
def test_conv_out_kernel_vs_torch(cuda, n, h, w, cin):
    """The RGB output conv (GroupNorm + SiLU + 3x3 conv to 3 channels + clamp / rescale, NCHW fp32) on 16 x 16
    LDS tiles over 32-channel chunks, including image sides that are not tile multiples."""
    C = __import__("dalle_amd.ops.ext", fromlist=["x"]).load_extension(required=True)
    torch.manual_seed(1)
    x = torch.randn(n, h, w, cin, device=cuda)
    conv = torch.nn.Conv2d(cin, 3, 3, 1, 1).to(cuda)
    norm = torch.nn.GroupNorm(32, cin, eps=1e-6).to(cuda)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.3, 0.3)
    xb = x.bfloat16().contiguous()
    ref = conv(torch.nn.functional.silu(norm(xb.float().permute(0, 3, 1, 2))))
    ref = (ref.clamp(-1, 1) + 1) * 0.5
    mean, rstd = C.gn_stats(xb, 1e-6)
    wk = conv.weight.detach().permute(0, 2, 3, 1).reshape(3, -1).bfloat16().contiguous()
    img = C.conv_out(xb, wk, conv.bias.detach().float(), mean, rstd, norm.weight.detach().float(), norm.bias.detach().float())
    assert img.shape == ref.shape
    assert (img - ref).abs().max().item() < 2e-2, (n, h, w, cin, (img - ref).abs().max().item())


def test_hip_decoder_matches_torch(cuda, monkeypatch):
    torch.manual_seed(0)
    ddconfig = dict(ch=128, out_ch=3, ch_mult=(1, 2, 4), num_res_blocks=1, attn_resolutions=(16,), resolution=64,
                    z_channels=256)
    vae = VQGanVAE(n_embed=512, embed_dim=256, ddconfig=ddconfig).to(cuda).eval()
    codes = torch.randint(0, 512, (3, 16 * 16), device=cuda)
    assert vae.use_hip_decoder()
    img = vae.decode(codes)
    monkeypatch.setattr(vae, "hip_decoder", False)
    ref = vae.decode(codes)
    assert img.shape == ref.shape == (3, 3, 64, 64)
    assert img.dtype == torch.float32 and img.min() >= 0 and img.max() <= 1
    err = (img - ref).abs()
    assert err.mean().item() < 1e-2 and _rel(img - 0.5, ref - 0.5) < 5e-2, (err.mean().item(), err.max().item())
