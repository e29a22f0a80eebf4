"""Parameter layouts (tensor shapes in State order) of the BASELINE.json configs."""
from __future__ import annotations

# examples/model-centric/01-Create-plan.ipynb:181-182 -- fc1 784->392, fc2 392->10
MNIST_SHAPES = [(392, 784), (392,), (10, 392), (10,)]


def resnet18_shapes(num_classes: int = 1000):
    """torchvision ResNet-18 ``model.parameters()`` order: 62 tensors, 11,689,512 params."""
    s = [(64, 3, 7, 7), (64,), (64,)]
    cin = 64
    for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
        for b in range(2):
            s += [(cout, cin if b == 0 else cout, 3, 3), (cout,), (cout,), (cout, cout, 3, 3), (cout,), (cout,)]
            if b == 0 and (stride != 1 or cin != cout):
                s += [(cout, cin, 1, 1), (cout,), (cout,)]
        cin = cout
    return s + [(num_classes, 512), (num_classes,)]


RESNET18_SHAPES = resnet18_shapes()
