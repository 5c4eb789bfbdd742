"""rtm — MI355X-native per-pixel ray-trace / ray-march renderer.

Drop-in for the CPU render loop of PtrMan/2018RustRayTracer (src/main.rs):
orthographic ray generation, ray-sphere front/back hits, fixed-step implicit
surface marching into a shadow map, Lambert + specular shading, RGBA
framebuffer write — as hand-written gfx950 HIP kernels behind a C ABI
(include/rtm.h, librtm.so).  The package name starts with a digit, so import it
with importlib.import_module("2018rustraytracer_amd").
"""
from . import abi, scenes  # noqa: F401
from .abi import RtmError, load_library  # noqa: F401
from .scenes import (Bilinear, Camera, EnumFace, Linear, PrimitiveCappedCylinder, PrimitiveCirclePlane,  # noqa: F401
                     PrimitiveSdf, PrimitiveSphere, Scene, Shading, eye_camera, perspective_eye_camera,
                     shadow_camera)
from .renderer import (Context, Group, HostRegistration, Viewport, device_count, encode_thresholds,  # noqa: F401
                       renderColorImage, render_frame, render_frame_ex, render_frame_multi, writeColorImage)
