from .stage1 import Stage1

__all__ = ["Stage1"]
