"""MI355X-native DDIM sampler for DiffPose (frame-based). See DESIGN.md."""
