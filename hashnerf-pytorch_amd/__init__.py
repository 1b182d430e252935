"""hashnerf_pytorch_amd -- MI355X (gfx950) drop-in for the HashNeRF hot path.

Module API mirrors mache102/HashNeRF-pytorch (HashEmbedder, SHEncoder,
NeRFSmall, render / render_rays / raw2outputs / sample_pdf, create_nerf,
RAdam, total_variation_loss); the arithmetic runs in the HIP C-ABI library
``lib/libhashnerf_amd.so`` (include/hashnerf_amd.h).  Import the package via
``hn_loader.load()`` (the directory name is not a Python identifier).
"""
from . import _lib
from .create import create_nerf
from .embedding import HashEmbedder, SHEncoder, hash, level_resolutions
from .loss import sigma_sparsity_loss, total_variation_loss, training_loss
from .models import NeRFSmall
from .radam import RAdam
from .rays import get_ndc_rays, get_rays, get_rays_np, pose_spherical
from .render import (NetworkQuery, batchify, img2mse, mse2psnr, raw2outputs, render, render_path,
                     render_rays, run_network, sample_pdf)

__all__ = ["HashEmbedder", "SHEncoder", "NeRFSmall", "RAdam", "create_nerf", "render", "render_rays",
           "render_path", "raw2outputs", "sample_pdf", "run_network", "batchify", "NetworkQuery",
           "total_variation_loss", "sigma_sparsity_loss", "training_loss", "get_rays", "get_rays_np", "get_ndc_rays",
           "pose_spherical", "img2mse", "mse2psnr", "hash", "level_resolutions"]
