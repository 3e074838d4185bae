"""MI355X-native PSO (Pairwise Sample Optimization) hot path for timestep-distilled SDXL.

Host side mirrors the reference's Python surface (pso_pytorch.diffusers_patch, the config_sdxl_*_dpo ConfigDicts,
and the diffusers UNet2DConditionModel call/checkpoint interface); all arithmetic runs in libpso_amd.so (HIP, gfx950).
"""
__version__ = "0.1.0"
