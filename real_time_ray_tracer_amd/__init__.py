"""MI355X-native per-pixel ray-scene intersection + shading hot path of
JustinPrivitera/Real_Time_Ray_Tracer (resources/{p,h,ao,aop}_compute.glsl,
aop_postprocessing.glsl) behind a C ABI (include/rt/abi.h, librtrt.so)."""
from ._lib import RtError, load  # noqa: F401
from .host import (AO_COMPUTE, AOP_COMPUTE, AOP_POSTPROCESSING, ASPECT_RATIO,  # noqa: F401
                   FULLSCREEN_ASPECT_RATIO, H_COMPUTE, P_COMPUTE, FrameDriver, GBuffer, Header,
                   Renderer, SSBO, StripGroup, aspect_for, header_floats, ssbo_floats)

__all__ = ["RtError", "load", "Renderer", "StripGroup", "Header", "SSBO", "GBuffer", "FrameDriver",
           "AOP_COMPUTE", "AOP_POSTPROCESSING", "AO_COMPUTE", "P_COMPUTE", "H_COMPUTE",
           "ASPECT_RATIO", "FULLSCREEN_ASPECT_RATIO", "aspect_for", "header_floats", "ssbo_floats"]
