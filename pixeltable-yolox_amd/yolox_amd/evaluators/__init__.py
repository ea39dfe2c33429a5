from .coco import COCOParams, coco_bbox_eval, convert_to_coco_format, summarize
from .coco_evaluator import CocoEvaluator, per_class_AP_table, per_class_AR_table, summary_text

__all__ = ["COCOParams", "CocoEvaluator", "coco_bbox_eval", "convert_to_coco_format", "per_class_AP_table",
           "per_class_AR_table", "summarize", "summary_text"]
