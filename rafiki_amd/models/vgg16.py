"""Vgg16 — VGG16 at 48x48x3 (the reference's TfVgg16, examples/models/image_classification/
TfVgg16.py:15-130): 13 conv3x3 layers (64,64 / 128,128 / 256x3 / 512x3 / 512x3, five 2x2 max-pools
48 -> 24 -> 12 -> 6 -> 3 -> 1), fc 4096 -> 4096 -> softmax, Adam, sparse cross-entropy; grayscale
inputs are stacked to three channels (TfVgg16.py:43).  Same knobs (epochs Fixed(1), learning_rate,
batch_size).

Runs on the gfx950 static-graph engine as the reference's network: conv3x3 + bias + ReLU blocks,
no BatchNorm (Keras VGG16, TfVgg16.py:115-130), 33.6 M parameters at 48x48x3 with 10 classes
(``ConvNetEngine(bn=False)``, fp32).  The ``batch_norm`` knob (default False) opts into the engine's
conv + BN + ReLU blocks instead.  The 48/24/12/6/3 maps use the implicit-GEMM conv's
reciprocal-decoded pixel gather (non-power-of-two extents), the 3 -> 1 pool the floor-mode odd
pooling path.
"""
import numpy as np

from rafiki_amd.constants import TaskType  # noqa: F401
from rafiki_amd.model import CategoricalKnob, FixedKnob, FloatKnob
from rafiki_amd.models.image_classifier import NativeImageClassifier

VGG16_CFG = (64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512, 'M')


class Vgg16(NativeImageClassifier):
    DEFAULT_IMAGE_SIZE = 48

    @staticmethod
    def get_knob_config():
        return {
            'epochs': FixedKnob(1),
            'learning_rate': FloatKnob(1e-5, 1e-2, is_exp=True),
            'batch_size': CategoricalKnob([16, 32, 64, 128]),
            'batch_norm': FixedKnob(False),
        }

    def _load(self, uri):
        images, labels, classes = super()._load(uri)
        if images.ndim == 3:
            images = np.stack([images] * 3, axis=-1)
        return images, labels, classes

    def _engine_kwargs(self, num_classes, channels, image_size):
        bn = bool(self._knobs.get('batch_norm', False))
        kw = dict(cfg=VGG16_CFG, fc_dims=(4096, 4096), optimizer='adam',
                  lr=float(self._knobs.get('learning_rate', 1e-3)), weight_decay=0.0, bn=bn)
        if not bn:
            kw['dtype'] = 'fp32'   # the conv + bias + ReLU blocks run on the fp32 engine
        return kw


if __name__ == '__main__':
    from rafiki_amd.model import test_model_class
    test_model_class(__file__, 'Vgg16', TaskType.IMAGE_CLASSIFICATION, {},
                     'synthetic://image?n=512&size=28&channels=1&classes=10&seed=0',
                     'synthetic://image?n=128&size=28&channels=1&classes=10&seed=1',
                     queries=[np.zeros((28, 28), np.uint8).tolist()],
                     knobs={'epochs': 1, 'learning_rate': 1e-3, 'batch_size': 32})
