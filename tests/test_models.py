"""Model zoo: parameter counts, checkpoint key contract, output signatures."""
import pytest
import torch

from pytorch_imageclassification_distributed_amd.models import (Classifier, efficientnet_b0, efficientnet_b3,
                                                                inception_v3, resnet18, resnet50, resnet101)


def nparams(m):
    return sum(p.numel() for p in m.parameters())


@pytest.mark.parametrize("ctor,expected", [
    (resnet18, 11_689_512), (resnet50, 25_557_032), (resnet101, 44_549_160),
    (inception_v3, 27_161_264), (efficientnet_b0, 5_288_548), (efficientnet_b3, 12_233_232),
])
def test_backbone_param_counts_match_published(ctor, expected):
    assert nparams(ctor()) == expected


@pytest.mark.parametrize("name,expected", [
    ("resnet18", 11_252_743), ("resnet50", 23_780_871), ("resnet101", 42_772_999),
    ("inceptionv3", 24_621_486), ("efficientnet-b0", 4_182_083), ("efficientnet-b3", 10_903_535),
])
def test_classifier_param_counts_7_classes(name, expected):
    assert nparams(Classifier(name, 7)) == expected


def test_resnet_state_dict_names():
    keys = set(Classifier("resnet50", 7).state_dict())
    for k in ["encoder.conv1.weight", "encoder.bn1.running_var", "encoder.bn1.num_batches_tracked",
              "encoder.layer1.0.conv1.weight", "encoder.layer1.0.downsample.0.weight",
              "encoder.layer1.0.downsample.1.bias", "encoder.layer4.2.bn3.weight",
              "encoder.fc.0.weight", "encoder.fc.2.weight", "encoder.fc.4.bias", "encoder.fc.6.weight"]:
        assert k in keys, k
    assert "encoder.fc.1.weight" not in keys  # ReLU at index 1


def test_inception_state_dict_names_and_outputs():
    m = Classifier("inceptionv3", 7)
    keys = set(m.state_dict())
    for k in ["encoder.Conv2d_1a_3x3.conv.weight", "encoder.Conv2d_1a_3x3.bn.running_mean",
              "encoder.Mixed_5b.branch5x5_2.conv.weight", "encoder.Mixed_6e.branch7x7dbl_5.bn.bias",
              "encoder.Mixed_7c.branch3x3dbl_3b.conv.weight", "encoder.AuxLogits.conv1.conv.weight",
              "encoder.AuxLogits.fc.weight", "encoder.fc.6.bias"]:
        assert k in keys, k
    assert m.encoder.AuxLogits.fc.out_features == 7
    x = torch.randn(2, 3, 299, 299)
    out = m(x)
    assert isinstance(out, tuple) and out[0].shape == (2, 7) and out[1].shape == (2, 7)
    m.eval()
    with torch.no_grad():
        assert m(x).shape == (2, 7)


def test_efficientnet_head_is_underscore_fc():
    m = Classifier("efficientnet-b0", 5)
    keys = set(m.state_dict())
    assert "encoder._fc.0.weight" in keys and "encoder._fc.6.bias" in keys
    assert "encoder._blocks.15._se_expand.bias" in keys
    assert "encoder._conv_head.weight" in keys
    assert m.encoder._bn0.momentum == pytest.approx(0.01) and m.encoder._bn0.eps == pytest.approx(1e-3)
    out = m(torch.randn(2, 3, 64, 64))
    assert out.shape == (2, 5)


def test_resnet18_cifar_shape_and_batch_constraint():
    m = Classifier("resnet18", 10)
    assert m(torch.randn(2, 3, 32, 32)).shape == (2, 10)


def test_unknown_model_raises():
    with pytest.raises(ValueError):
        Classifier("vgg16", 7)


def test_pretrained_local_state_dict(tmp_path):
    src = resnet18()
    p = tmp_path / "r18.pth"
    torch.save(src.state_dict(), p)
    m = Classifier("resnet18", 7, pretrained=str(p))
    assert torch.equal(m.encoder.conv1.weight, src.conv1.weight)
