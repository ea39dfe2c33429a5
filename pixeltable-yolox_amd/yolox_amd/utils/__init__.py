from .boxes import (bboxes_iou, cxcywh2xyxy, postprocess, postprocess_device, xyxy2cxcywh,  # noqa: F401
                    xyxy2xywh)
