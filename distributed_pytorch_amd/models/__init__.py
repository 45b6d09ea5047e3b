from .vgg import CFG, VGG, VGG11, VGG13, VGG16, VGG19, VGGSpec, make_layers  # noqa: F401
