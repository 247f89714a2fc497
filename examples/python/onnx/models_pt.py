"""The torch models the reference ONNX examples export (examples/python/onnx/*_pt.py; AlexNet and
ResNet are the torchvision definitions, written out because torchvision is not installed)."""
import torch
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.linear1 = nn.Linear(784, 512)
        self.linear2 = nn.Linear(512, 512)
        self.linear3 = nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=1)

    def forward(self, x):
        y = self.relu(self.linear1(x))
        y = self.relu(self.linear2(y))
        return self.softmax(self.linear3(y))


class CNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3)
        self.conv2 = nn.Conv2d(32, 32, 3)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv3 = nn.Conv2d(32, 64, 3)
        self.conv4 = nn.Conv2d(64, 64, 3)
        self.linear1 = nn.Linear(64 * 5 * 5, 512)
        self.linear2 = nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=1)

    def forward(self, x):
        y = self.pool(self.relu(self.conv2(self.relu(self.conv1(x)))))
        y = self.pool(self.relu(self.conv4(self.relu(self.conv3(y)))))
        y = torch.flatten(y, 1)
        return self.softmax(self.linear2(self.relu(self.linear1(y))))


class AlexNet(nn.Module):
    def __init__(self, num_classes=10, size=224):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, kernel_size=11, stride=4, padding=2), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2),
            nn.Conv2d(64, 192, kernel_size=5, padding=2), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2),
            nn.Conv2d(192, 384, kernel_size=3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(256, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2))
        with torch.no_grad():  # 256 x 6 x 6 at 224 / 229 px, smaller for the CPU-test sizes
            flat = self.features(torch.zeros(1, 3, size, size)).numel()
        self.classifier = nn.Sequential(
            nn.Linear(flat, 4096), nn.ReLU(inplace=True), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes), nn.Softmax(dim=1))

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        identity = x if self.down is None else self.down(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out += identity
        return self.relu(out)


class ResNet18(nn.Module):
    def __init__(self, num_classes=10, widths=(64, 128, 256, 512)):
        super().__init__()
        self.conv1 = nn.Conv2d(3, widths[0], 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(widths[0])
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        layers, cin = [], widths[0]
        for i, w in enumerate(widths):
            layers += [BasicBlock(cin, w, 1 if i == 0 else 2), BasicBlock(w, w)]
            cin = w
        self.layers = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.avgpool(self.layers(x))
        return self.fc(torch.flatten(x, 1))
