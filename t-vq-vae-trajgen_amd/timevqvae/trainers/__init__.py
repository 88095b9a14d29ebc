"""Lightning-free Stage1 / Stage2 / Stage3 trainers over the HIP modules (reference trainers/)."""
from .stage1 import Stage1
from .stage2 import Stage2
from .stage3 import Stage3

__all__ = ["Stage1", "Stage2", "Stage3"]
