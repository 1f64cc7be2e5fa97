"""MI355X-native (gfx950 / CDNA4) distributed image-classification trainer.

Capabilities of RanjanBalappa/pytorch-imageclassification-distributed (see
SURVEY.md), re-designed MI355X-first:

* ``models``   ResNet-18/34/50/101/152, Inception-v3 (+aux), EfficientNet-B0..B7
               behind ``Classifier(name, num_classes)`` with the reference MLP head.
* ``ops``      functional op layer; GPU path = hand-written HIP kernels in
               ``csrc/`` (MFMA implicit-GEMM conv, fused BN/ReLU/residual,
               pooling, loss, Adam), CPU path = ATen reference.
* ``parallel`` process group (RCCL over xGMI / gloo), bucketed gradient
               all-reduce overlapped with backward, SyncBatchNorm, object
               all-gather.
* ``data``     ImageFolder-style augmented dataset, synthetic on-device data,
               H2D prefetcher.
* ``engine``   trainer loop with the reference semantics, checkpoint/resume.
"""
__version__ = "0.1.0"
