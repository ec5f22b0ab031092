"""ap_gym_amd — MI355X (gfx950) backend for ap_gym's data-parallel hot path.

    import ap_gym_amd as ap
    env = ap.make_vec("LIDARLocRooms-v0", num_envs=65536, lidar_beam_count=32,
                      dataset=ap.FloorMapDatasetRooms(64, 64), array_backend="torch")
    obs, info = env.reset(seed=0)
    obs, reward, terminated, truncated, info = env.step({"action": a, "prediction": p})

The compute path is the HIP library _lib/libapgym_hip.so (C ABI: include/apgym_capi.h); there is
no CPU fallback.
"""

from . import _native  # noqa: F401
from .circle_square import (  # noqa: F401
    CircleSquareDataset,
    CircleSquareHideAndSeekVectorWrapper,
    DoubleCircleSquareDataset,
)
from .floor_map import (ArrayFloorMapDataset, FloorMapDataset, FloorMapDatasetMaze, FloorMapDatasetRooms,  # noqa: F401
                        ForeignFloorMapView, PoolFloorMapDataset)
from .image_dataset import (  # noqa: F401
    ArrayImageClassificationDataset,
    HuggingfaceImageClassificationDataset,
    ImageClassificationDataset,
    SyntheticImageClassificationDataset,
)
from .image_env import ImageClassificationVectorEnv, ImageLocalizationVectorEnv, ImagePerceptionConfig  # noqa: F401
from .lidar_env import LIDARLocalization2DVectorEnv, lidar_beam_directions  # noqa: F401
from .light_dark_env import LightDarkVectorEnv  # noqa: F401
from .loss_fn import (  # noqa: F401
    CrossEntropyLossFn,
    LambdaLossFn,
    LossFn,
    LossFnAffineTransformation,
    MSELossFn,
    WeightedLossFn,
    ZeroLossFn,
)
from .registration import make_vec, register, registry  # noqa: F401
from .spaces import ActivePerceptionActionSpace, ImageSpace, LogitSpace  # noqa: F401

__version__ = "0.1.0"
