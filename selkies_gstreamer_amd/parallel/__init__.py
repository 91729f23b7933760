"""Multi-GPU / multi-session parallelism: placement, node launcher, RCCL packet fan-in."""
