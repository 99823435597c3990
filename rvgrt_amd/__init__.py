"""rvgrt_amd -- MI355X-native voxel ray-tracing render path.

A drop-in for RubenVlieger/RVGRT's CUDA render path (StateRender::drawCUDA
and the raytracing_functions it calls), rebuilt as hand-written HIP kernels
for gfx950 behind the C ABI in include/rvgrt.h (librvgrt_hip.so).
"""
from . import _lib
from ._lib import (RV_F_GI, RV_F_PREPASS, RV_F_REF_FETCH, RV_F_SHADOW, RV_F_STATS, RV_F_WATER,
                   RV_FLAGS_REFERENCE, RV_IMAGE_COLOR, RV_IMAGE_DEPTH, RV_IMAGE_HALF_DIST,
                   RV_IMAGE_HALF_SHADOW, RV_IMAGE_MOTION, RV_WORLD_BITS, RV_WORLD_CSDF,
                   RV_WORLD_GI, RvError, RV_OPT_PIPE_ORDER, RV_OPT_BATCH_STREAMS, RV_OPT_FLOW_SPIN,
                   RV_OPT_FLOW_FORCE_FALLBACK, RV_OPT_GI_PAIRS, RV_OPT_GI_SHARD_PROBE, RV_EXIT_SKY,
                   RV_EXIT_COLUMN, RV_EXIT_SUN)
from .configs import CONFIGS, RenderConfig
from .render import Comm, LoopbackGroup, StateRender, camera_dict, camera_from_pose, frame_desc

__all__ = ["StateRender", "Comm", "LoopbackGroup", "camera_from_pose", "camera_dict", "frame_desc", "CONFIGS", "RenderConfig", "RvError",
           "RV_F_GI", "RV_F_PREPASS", "RV_F_REF_FETCH", "RV_F_SHADOW", "RV_F_STATS", "RV_F_WATER",
           "RV_FLAGS_REFERENCE", "RV_IMAGE_COLOR", "RV_IMAGE_DEPTH", "RV_IMAGE_HALF_DIST",
           "RV_IMAGE_HALF_SHADOW", "RV_IMAGE_MOTION", "RV_WORLD_BITS", "RV_WORLD_CSDF",
           "RV_WORLD_GI", "_lib"]
