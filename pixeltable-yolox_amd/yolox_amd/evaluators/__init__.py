from .coco import COCOParams, coco_bbox_eval, convert_to_coco_format, summarize

__all__ = ["COCOParams", "coco_bbox_eval", "convert_to_coco_format", "summarize"]
