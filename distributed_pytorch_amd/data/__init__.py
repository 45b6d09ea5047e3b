from .cifar import (MEAN, STD, DeviceLoader, ImageSet, ShardSampler, get_datasets, load_cifar10,  # noqa: F401
                    synthetic_cifar)
