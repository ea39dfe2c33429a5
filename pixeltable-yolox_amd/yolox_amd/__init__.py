"""yolox_amd -- MI355X-native YOLOX hot path (drop-in for pixeltable-yolox's
yolox.models.Yolox / YoloxModule / YoloxProcessor and yolox.utils.postprocess)."""
from .config import YoloxConfig  # noqa: F401

__version__ = "0.1.0"
