"""BASELINE config 1: infer.py with the 'big' preset, CPU-only PyTorch, on data_test/catstatue_rgba.png, one 256^2
render -- the plumbing run. The reference cannot run it: core/gs.py:20 puts the background on "cuda"
and its rasterizer is CUDA-only; MVDream / rembg need network (infer.py:58-67). This harness runs the reference's
own flow with lgm_amd's modules swapped in:

  * the UNet is the reference's core/unet.py UNet('big': core/options.py:96-107 -> up_channels (1024, 1024, 512,
    256, 128), up_attention (T, T, T, F, F)), imported from the reference checkout (out of scope: stock convs), with
    every one of its 16 MVAttention blocks replaced by lgm_amd.attention.MVAttention loaded from the block's own
    state_dict (strict) -- on CPU tensors that module takes lgm_amd/cpu.py's torch path;
  * infer.py:70-104's input: the RGBA PNG composited on white (:83-84), replicated to the 4 views that MVDream would
    generate (the substitution SURVEY §3.2 prescribes: no network), resized to input_size (:96), ImageNet-normalised
    (:97) and concatenated with the default Pluecker rays (core/models.py:61-85, lgm_amd.cameras.default_rays);
    kiui's recenter (:79) is skipped (the PNG is already cut out and centred);
  * forward_gaussians' epilogue (core/models.py:96-117) by lgm_amd.head.gaussian_head (CPU: torch ops);
  * save_ply (infer.py:107) and ONE orbit render at 256^2 (infer.py:134-145's first frame) by
    lgm_amd.GaussianRenderer on CPU tensors (lgm_amd/cpu.py).
fp32 throughout (infer.py:44 casts to half for CUDA; half convolutions are not a CPU path). Random init: no
checkpoint exists offline (infer.py:32-40 warns the same way).

    python scripts/cfg1_cpu.py [--reference /root/reference] [--png tests/golden/catstatue_rgba.png] [--threads N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

BIG = dict(down_channels=(64, 128, 256, 512, 1024, 1024), down_attention=(False, False, False, True, True, True),
           mid_attention=True, up_channels=(1024, 1024, 512, 256, 128), up_attention=(True, True, True, False, False))
INPUT_SIZE, SPLAT_SIZE, RENDER_SIZE = 256, 128, 256
IMAGENET_MEAN, IMAGENET_STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


def build_big_unet(reference_root: str):
    """The reference's UNet('big') with lgm_amd's MVAttention swapped in; returns (unet, number of swapped blocks)."""
    if reference_root not in sys.path:
        sys.path.insert(0, reference_root)
    os.environ.setdefault("XFORMERS_DISABLED", "1")  # xformers is absent; every attention block is swapped anyway
    sys.dont_write_bytecode = True  # the reference checkout is read-only
    from core.unet import MVAttention as RefMVA
    from core.unet import UNet

    from lgm_amd.attention import MVAttention
    unet = UNet(9, 14, **BIG)
    swapped = 0
    for parent in list(unet.modules()):
        for name, child in list(parent.named_children()):
            if isinstance(child, RefMVA):
                mine = MVAttention(child.norm.num_channels, child.attn.num_heads, residual=child.residual,
                                   skip_scale=child.skip_scale, num_frames=child.num_frames,
                                   groups=child.norm.num_groups, eps=child.norm.eps,
                                   qkv_bias=child.attn.qkv.bias is not None,
                                   proj_bias=child.attn.proj.bias is not None)
                mine.load_state_dict(child.state_dict(), strict=True)
                setattr(parent, name, mine)
                swapped += 1
    return unet, swapped


def load_views(png: str, size: int = INPUT_SIZE) -> torch.Tensor:
    """infer.py:70-99 without rembg / recenter / MVDream: [1, 4, 9, size, size] (RGB normalised + rays)."""
    from PIL import Image

    from lgm_amd.cameras import default_rays
    img = np.asarray(Image.open(png).convert("RGBA")).astype(np.float32) / 255.0  # [H, W, 4]
    rgb = img[..., :3] * img[..., 3:4] + (1 - img[..., 3:4])  # white background (infer.py:83-84)
    mv = np.stack([rgb] * 4, axis=0)  # the 4 views MVDream would generate
    x = torch.from_numpy(mv).permute(0, 3, 1, 2).float()
    x = F.interpolate(x, size=(size, size), mode="bilinear", align_corners=False)
    mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    x = (x - mean) / std
    return torch.cat([x, default_rays(size)], dim=1).unsqueeze(0)


def run(reference_root: str, png: str, out_dir: str, threads: int = 0, seed: int = 0) -> dict:
    from lgm_amd import GaussianRenderer, Options
    from lgm_amd.cameras import cameras_from_c2w, orbit_camera, projection_matrix
    from lgm_amd.head import GaussianHead
    if threads > 0:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    t = {}
    t0 = time.perf_counter()
    unet, swapped = build_big_unet(reference_root)
    head = GaussianHead()  # LGM.conv (core/models.py:34) + the activations
    unet.eval()
    t["build_s"] = time.perf_counter() - t0
    images = load_views(png)
    B, V = images.shape[:2]
    opt = Options(input_size=INPUT_SIZE, splat_size=SPLAT_SIZE, output_size=RENDER_SIZE)
    renderer = GaussianRenderer(opt)
    with torch.no_grad():
        t0 = time.perf_counter()
        feats = unet(images.view(B * V, 9, INPUT_SIZE, INPUT_SIZE))  # [4, 14, 128, 128]
        t["unet_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        gaussians = head(feats, B, V)  # [1, 4 * 128^2, 14]
        t["head_s"] = time.perf_counter() - t0
        os.makedirs(out_dir, exist_ok=True)
        renderer.save_ply(gaussians, os.path.join(out_dir, "catstatue.ply"))
        pose = torch.from_numpy(orbit_camera(0, 0, radius=opt.cam_radius, opengl=True)).unsqueeze(0)
        cv, cvp, cp = cameras_from_c2w(pose, projection_matrix(opt.fovy, opt.znear, opt.zfar))
        t0 = time.perf_counter()
        out = renderer.render(gaussians, cv[None], cvp[None], cp[None], scale_modifier=1)
        t["render_s"] = time.perf_counter() - t0
    frame = (out["image"].squeeze(1).permute(0, 2, 3, 1).contiguous().float().numpy() * 255).astype(np.uint8)
    return {"config": "cfg1: infer.py 'big', CPU-only, data_test/catstatue_rgba.png, 1 view 256^2",
            "swapped_mvattention_blocks": swapped, "unet_out": list(feats.shape), "gaussians": list(gaussians.shape),
            "frame": list(frame.shape), "alpha_mean": float(out["alpha"].mean()),
            "image_finite": bool(torch.isfinite(out["image"]).all()), "threads": torch.get_num_threads(),
            "seconds": {k: round(v, 3) for k, v in t.items()}, "_frame": frame}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--png", default=os.path.join(ROOT, "tests", "golden", "catstatue_rgba.png"))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cfg1"))
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    res = run(a.reference, a.png, a.out, a.threads)
    res.pop("_frame")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
