"""rvcp-real-time-path-tracer_amd -- MI355X-native drop-in for the path-tracing hot path of
YXHXianYu/RVCP-Real-Time-Path-Tracer (assets/shaders/ray_tracer_games101_branch.comp).

The package directory name contains hyphens, so import it through ``rvcp_amd.py`` at the
repository root (``import rvcp_amd``), which loads this package under the name ``rvcp_amd``.
"""
from . import abi, scene
from .scene import (Camera, Face, Material, MaterialType, Mesh, Scene, Sphere, Vertex,
                    cornell_box, push_constant)
from .ray_tracer import RayTracer, rccl_unique_id, shard_row_ids, shard_rows
from . import frame
from . import interactive
from . import scene_io
from . import mandelbrot

__all__ = ["abi", "scene", "frame", "interactive", "scene_io", "mandelbrot", "Camera", "Face", "Material", "MaterialType", "Mesh", "Scene",
           "Sphere", "Vertex", "cornell_box", "push_constant", "RayTracer", "rccl_unique_id",
           "shard_rows", "shard_row_ids"]
