"""Parameter-list sizes of the reference's CIFAR-10 models, in registration
order, for synthetic per-tensor gradient lists (no model code is needed: the
reducers only see the list of gradient tensors).

    resnet50_sizes()  161 tensors, 23,520,842 elements  (models/resnet.py ResNet50)
    vgg16_sizes()      54 tensors, 14,728,266 elements  (models/vgg.py VGG16)

These are the bucket sizes SURVEY.md §8(d) quotes for configs 3 and 4.
"""
from __future__ import annotations


def resnet50_sizes(num_classes: int = 10) -> list[int]:
    sizes: list[int] = []

    def conv(cin, cout, k):
        sizes.append(cout * cin * k * k)

    def bn(c):
        sizes.extend([c, c])

    conv(3, 64, 3)
    bn(64)
    inp = 64
    for planes, blocks, stride in [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]:
        for b in range(blocks):
            s = stride if b == 0 else 1
            conv(inp, planes, 1)
            bn(planes)
            conv(planes, planes, 3)
            bn(planes)
            conv(planes, 4 * planes, 1)
            bn(4 * planes)
            if s != 1 or inp != 4 * planes:
                conv(inp, 4 * planes, 1)
                bn(4 * planes)
            inp = 4 * planes
    sizes += [num_classes * 2048, num_classes]
    return sizes


def vgg16_sizes(num_classes: int = 10) -> list[int]:
    cfg = [64, 64, 128, 128, 256, 256, 256, 512, 512, 512, 512, 512, 512]
    sizes: list[int] = []
    inp = 3
    for v in cfg:
        sizes += [v * inp * 9, v, v, v]  # conv weight, conv bias, bn weight, bn bias
        inp = v
    sizes += [num_classes * 512, num_classes]
    return sizes
