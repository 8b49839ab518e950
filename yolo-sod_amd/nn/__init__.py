from .modules import *  # noqa: F401,F403
from .tasks import DetectionModel, build_model, parse_model, yaml_model_load  # noqa: F401
