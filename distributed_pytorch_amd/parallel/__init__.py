from .comm import Comm, NullComm, RcclComm, TorchComm  # noqa: F401
from .launch import DistContext, env_dict, init_cli, init_env, init_single  # noqa: F401
from .sync import (DEFAULT_BUCKET_MB, MODES, AllReduceSync, DDPSync, GatherScatterSync, GradSync,  # noqa: F401
                   make_sync, plan_buckets)
