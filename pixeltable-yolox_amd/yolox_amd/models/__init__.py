from .network import (BaseConv, Bottleneck, CspDarknet, CspLayer, DWConv, Focus,  # noqa: F401
                      SPPBottleneck, YoloPafpn, YoloxHead)
from .processor import Detections, YoloxProcessor  # noqa: F401
from .yolox import Yolox, YoloxModule  # noqa: F401
