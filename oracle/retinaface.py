"""RetinaFace-ResNet50 + FPN + SSH + heads forward on torch-CPU fp32 — the
floating-point reference for the HIP conv path. Test infrastructure only.

Module tree and state_dict keys follow the reference exactly so a converted
reference checkpoint loads into both this oracle and the HIP library:
* ``body``  = torchvision resnet50 wrapped by IntermediateLayerGetter
  (detect_face/retinaface.py:71-73 [ext]; v1.5 bottleneck, stride on the 3x3;
  returns layer2/3/4, config.py:26; fc/avgpool dropped);
* ``fpn``   = FPN (detect_face/nets/layers.py:68-114; leaky=0 since out=256>64, :71);
* ``ssh1..3`` = SSH (layers.py:37-66);
* ``ClassHead/BboxHead/LandmarkHead`` ModuleLists (retinaface.py:13-51,90-92).
Eval forward returns (loc, softmax(conf), landm) (retinaface.py:114-148) and,
for parity on raw logits, ``forward_raw`` returns the un-softmaxed class logits.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return self.relu(out + idt)


class ResNet50Body(nn.Module):
    """torchvision.models.resnet50 up to layer4 [ext]."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.inplanes = 64
        self.layer1 = self._make(64, 3, 1)
        self.layer2 = self._make(128, 4, 2)
        self.layer3 = self._make(256, 6, 2)
        self.layer4 = self._make(512, 3, 2)

    def _make(self, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        c2 = self.layer1(x)
        c3 = self.layer2(c2)
        c4 = self.layer3(c3)
        c5 = self.layer4(c4)
        return [c3, c4, c5]


def conv_bn(inp, oup, stride=1, leaky=0.0):           # layers.py:10-15
    return nn.Sequential(nn.Conv2d(inp, oup, 3, stride, 1, bias=False), nn.BatchNorm2d(oup),
                         nn.LeakyReLU(negative_slope=leaky, inplace=True))


def conv_bn1x1(inp, oup, stride, leaky=0.0):         # layers.py:17-22
    return nn.Sequential(nn.Conv2d(inp, oup, 1, stride, 0, bias=False), nn.BatchNorm2d(oup),
                         nn.LeakyReLU(negative_slope=leaky, inplace=True))


def conv_bn_no_relu(inp, oup, stride):               # layers.py:28-32
    return nn.Sequential(nn.Conv2d(inp, oup, 3, stride, 1, bias=False), nn.BatchNorm2d(oup))


class SSH(nn.Module):                                # layers.py:37-66
    def __init__(self, cin, cout):
        super().__init__()
        leaky = 0.1 if cout <= 64 else 0
        self.conv3X3 = conv_bn_no_relu(cin, cout // 2, 1)
        self.conv5X5_1 = conv_bn(cin, cout // 4, 1, leaky)
        self.conv5X5_2 = conv_bn_no_relu(cout // 4, cout // 4, 1)
        self.conv7X7_2 = conv_bn(cout // 4, cout // 4, 1, leaky)
        self.conv7x7_3 = conv_bn_no_relu(cout // 4, cout // 4, 1)

    def forward(self, x):
        c3 = self.conv3X3(x)
        c5_1 = self.conv5X5_1(x)
        c5 = self.conv5X5_2(c5_1)
        c7_2 = self.conv7X7_2(c5_1)
        c7 = self.conv7x7_3(c7_2)
        return F.relu(torch.cat([c3, c5, c7], 1))


class FPN(nn.Module):                                # layers.py:68-114
    def __init__(self, in_list, cout):
        super().__init__()
        leaky = 0.1 if cout <= 64 else 0
        self.output1 = conv_bn1x1(in_list[0], cout, 1, leaky)
        self.output2 = conv_bn1x1(in_list[1], cout, 1, leaky)
        self.output3 = conv_bn1x1(in_list[2], cout, 1, leaky)
        self.merge1 = conv_bn(cout, cout, leaky=leaky)
        self.merge2 = conv_bn(cout, cout, leaky=leaky)

    def forward(self, xs):
        o1 = self.output1(xs[0])
        o2 = self.output2(xs[1])
        o3 = self.output3(xs[2])
        o2 = self.merge2(o2 + F.interpolate(o3, size=[o2.size(2), o2.size(3)], mode="nearest"))
        o1 = self.merge1(o1 + F.interpolate(o2, size=[o1.size(2), o1.size(3)], mode="nearest"))
        return [o1, o2, o3]


class _Head(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1x1 = nn.Conv2d(cin, cout, 1, 1, 0)


class RetinaFaceR50(nn.Module):
    """retinaface.py:53-148 with cfg_re50 (in_channel 256, out_channel 256)."""

    def __init__(self):
        super().__init__()
        self.body = ResNet50Body()
        self.fpn = FPN([512, 1024, 2048], 256)
        self.ssh1 = SSH(256, 256)
        self.ssh2 = SSH(256, 256)
        self.ssh3 = SSH(256, 256)
        self.ClassHead = nn.ModuleList([_Head(256, 4) for _ in range(3)])
        self.BboxHead = nn.ModuleList([_Head(256, 8) for _ in range(3)])
        self.LandmarkHead = nn.ModuleList([_Head(256, 20) for _ in range(3)])

    def features(self, x):
        fpn = self.fpn(self.body(x))
        return [self.ssh1(fpn[0]), self.ssh2(fpn[1]), self.ssh3(fpn[2])]

    @staticmethod
    def _flat(conv, f, k):
        out = conv(f).permute(0, 2, 3, 1).contiguous()
        return out.view(out.shape[0], -1, k)

    def forward_raw(self, x):
        feats = self.features(x)
        loc = torch.cat([self._flat(self.BboxHead[i].conv1x1, f, 4) for i, f in enumerate(feats)], 1)
        cls = torch.cat([self._flat(self.ClassHead[i].conv1x1, f, 2) for i, f in enumerate(feats)], 1)
        ldm = torch.cat([self._flat(self.LandmarkHead[i].conv1x1, f, 10) for i, f in enumerate(feats)], 1)
        return loc, cls, ldm

    def forward(self, x):
        loc, cls, ldm = self.forward_raw(x)
        return loc, F.softmax(cls, dim=-1), ldm


def _dw(inp, oup, stride):                             # mobilenet025.py:10-19 (conv_dw)
    return nn.Sequential(nn.Conv2d(inp, inp, 3, stride, 1, groups=inp, bias=False), nn.BatchNorm2d(inp),
                         nn.LeakyReLU(negative_slope=0.1, inplace=True),
                         nn.Conv2d(inp, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup),
                         nn.LeakyReLU(negative_slope=0.1, inplace=True))


class MobileNetV1Body(nn.Module):
    """mobilenet025.py:21-48 up to stage3, returning stage1/2/3 (cfg_mnet
    return_layers, config.py:1-16): 64/128/256 channels at strides 8/16/32."""

    def __init__(self):
        super().__init__()
        self.stage1 = nn.Sequential(conv_bn(3, 8, 2, leaky=0.1), _dw(8, 16, 1), _dw(16, 32, 2), _dw(32, 32, 1),
                                    _dw(32, 64, 2), _dw(64, 64, 1))
        self.stage2 = nn.Sequential(_dw(64, 128, 2), *[_dw(128, 128, 1) for _ in range(5)])
        self.stage3 = nn.Sequential(_dw(128, 256, 2), _dw(256, 256, 1))

    def forward(self, x):
        s1 = self.stage1(x)
        s2 = self.stage2(s1)
        return [s1, s2, self.stage3(s2)]


class RetinaFaceMnet(RetinaFaceR50):
    """retinaface.py:53-148 with cfg_mnet (in_channel 32, out_channel 64)."""

    def __init__(self):
        nn.Module.__init__(self)
        self.body = MobileNetV1Body()
        self.fpn = FPN([64, 128, 256], 64)
        self.ssh1 = SSH(64, 64)
        self.ssh2 = SSH(64, 64)
        self.ssh3 = SSH(64, 64)
        self.ClassHead = nn.ModuleList([_Head(64, 4) for _ in range(3)])
        self.BboxHead = nn.ModuleList([_Head(64, 8) for _ in range(3)])
        self.LandmarkHead = nn.ModuleList([_Head(64, 20) for _ in range(3)])


def build_oracle_model(state_dict):
    """Instantiate the oracle network from a reference-keyed state_dict
    (numpy arrays or tensors); body.stage1.* keys select the MobileNet-0.25
    model (the reference's backbone="mobilenet", retinaface.py:60)."""
    m = (RetinaFaceMnet() if "body.stage1.0.0.weight" in state_dict else RetinaFaceR50()).eval()
    sd = {k: torch.as_tensor(v) for k, v in state_dict.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("num_batches_tracked")]
    if missing or unexpected:
        raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    return m
