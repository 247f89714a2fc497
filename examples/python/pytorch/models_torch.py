"""Torch model definitions of the reference pytorch examples (torchvision / classy_vision are not
installed, so ResNet, SqueezeNet and a RegNetX are written out here; CNN is the reference's
two-input cifar10 model, examples/python/pytorch/cifar10_cnn_torch.py)."""
import torch
import torch.nn as nn


class CNN(nn.Module):
    """Two inputs through a shared conv, concatenated, split and re-joined (reference CNN)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, 1)
        self.conv2 = nn.Conv2d(64, 32, 3, 1)
        self.pool1 = nn.MaxPool2d(2, 2)
        self.conv3 = nn.Conv2d(32, 64, 3, 1)
        self.conv4 = nn.Conv2d(64, 64, 3, 1)
        self.pool2 = nn.MaxPool2d(2, 2)
        self.flat1 = nn.Flatten()
        self.linear1 = nn.Linear(64 * 5 * 5, 512)
        self.linear2 = nn.Linear(512, 10)
        self.relu = nn.ReLU()

    def forward(self, input1, input2):
        y1 = self.relu(self.conv1(input1))
        y2 = self.relu(self.conv1(input2))
        y = torch.cat((y1, y2), 1)
        (y1, y2) = torch.split(y, 32, 1)
        y = torch.cat((y1, y2), 1)
        y = self.pool1(self.relu(self.conv2(y)))
        y = self.relu(self.conv4(self.relu(self.conv3(y))))
        y = self.flat1(self.pool2(y))
        y = self.relu(self.linear1(y))
        return (self.linear2(y), y)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != planes:
            self.downsample = nn.Sequential(nn.Conv2d(cin, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out += identity
        return self.relu(out)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != planes * 4:
            self.downsample = nn.Sequential(nn.Conv2d(cin, planes * 4, 1, stride, bias=False),
                                            nn.BatchNorm2d(planes * 4))

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        out += identity
        return self.relu(out)


class ResNet(nn.Module):
    """torchvision's ResNet layout (7x7/2 stem, max pool, four stages, global pool, fc)."""

    def __init__(self, block, layers, num_classes=1000, width=64):
        super().__init__()
        self.inplanes = width
        self.conv1 = nn.Conv2d(3, width, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, width, layers[0], 1)
        self.layer2 = self._make(block, width * 2, layers[1], 2)
        self.layer3 = self._make(block, width * 4, layers[2], 2)
        self.layer4 = self._make(block, width * 8, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(width * 8 * block.expansion, num_classes)

    def _make(self, block, planes, n, stride):
        layers = [block(self.inplanes, planes, stride)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, n)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(num_classes=1000, width=64):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, width)


def resnet152(num_classes=1000, width=64):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, width)


class Fire(nn.Module):
    def __init__(self, cin, squeeze, e1, e3):
        super().__init__()
        self.squeeze = nn.Conv2d(cin, squeeze, 1)
        self.expand1x1 = nn.Conv2d(squeeze, e1, 1)
        self.expand3x3 = nn.Conv2d(squeeze, e3, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        x = self.relu(self.squeeze(x))
        return torch.cat([self.relu(self.expand1x1(x)), self.relu(self.expand3x3(x))], 1)


class SqueezeNet(nn.Module):
    """torchvision squeezenet1_1 layout (reference examples/python/pytorch/torch_vision_torch.py)."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 3, 2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            Fire(64, 16, 64, 64), Fire(128, 16, 64, 64), nn.MaxPool2d(3, 2),
            Fire(128, 32, 128, 128), Fire(256, 32, 128, 128), nn.MaxPool2d(3, 2),
            Fire(256, 48, 192, 192), Fire(384, 48, 192, 192), Fire(384, 64, 256, 256), Fire(512, 64, 256, 256))
        self.classifier = nn.Sequential(nn.Dropout(p=0.5), nn.Conv2d(512, num_classes, 1), nn.ReLU(inplace=True),
                                        nn.AdaptiveAvgPool2d((1, 1)))

    def forward(self, x):
        return torch.flatten(self.classifier(self.features(x)), 1)


class XBlock(nn.Module):
    """RegNetX bottleneck: 1x1, grouped 3x3, 1x1, residual (reference export_regnet_fx.py used
    classy_vision's RegNetX32gf; this is the same block family at configurable widths)."""

    def __init__(self, cin, cout, stride, group_width):
        super().__init__()
        self.a = nn.Sequential(nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))
        self.b = nn.Sequential(nn.Conv2d(cout, cout, 3, stride, 1, groups=cout // group_width, bias=False),
                               nn.BatchNorm2d(cout), nn.ReLU(inplace=True))
        self.c = nn.Sequential(nn.Conv2d(cout, cout, 1, bias=False), nn.BatchNorm2d(cout))
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        s = x if self.proj is None else self.proj(x)
        return self.relu(self.c(self.b(self.a(x))) + s)


class RegNetX(nn.Module):
    def __init__(self, depths=(2, 4, 8, 2), widths=(96, 192, 432, 1008), group_width=48, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True))
        blocks, cin = [], 32
        for d, w in zip(depths, widths):
            for i in range(d):
                blocks.append(XBlock(cin, w, 2 if i == 0 else 1, group_width))
                cin = w
        self.trunk = nn.Sequential(*blocks)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        return self.fc(torch.flatten(self.avgpool(self.trunk(self.stem(x))), 1))
