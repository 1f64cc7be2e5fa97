from .checkpoint import (BEST, LATEST, ddp_state_dict, load_checkpoint, load_model_state,
                         resolve_resume, restore_rng_state, save_checkpoint)
from .meters import Accuracy, AccuracyCounter, AverageMeter, DeviceMeter
from .timers import JsonlLogger, PhaseTimer

__all__ = [
    "AverageMeter", "Accuracy", "DeviceMeter", "AccuracyCounter",
    "save_checkpoint", "load_checkpoint", "load_model_state", "resolve_resume", "ddp_state_dict",
    "restore_rng_state",
    "BEST", "LATEST", "PhaseTimer", "JsonlLogger",
]
