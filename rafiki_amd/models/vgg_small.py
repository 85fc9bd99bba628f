"""VggSmall — the BASELINE benchmark model (VGG-small 32x32x3, conv3x3+BN+ReLU stacks) as a
Rafiki model.  Upload this file with ``Client.create_model(..., model_class='VggSmall')``.

Reference analogue: examples/models/image_classification/TfVgg16.py (Keras VGG16 at 48x48x3,
Adam, knobs epochs/learning_rate/batch_size).  Runs on the gfx950 static-graph engine
(``rafiki_amd.engine.convnet``) on GPU, and on its PyTorch reference path on CPU.
"""
from rafiki_amd.constants import TaskType  # noqa: F401
from rafiki_amd.engine.convnet import VGG_SMALL_CFG
from rafiki_amd.model import CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob
from rafiki_amd.models.image_classifier import NativeImageClassifier


class VggSmall(NativeImageClassifier):
    DEFAULT_IMAGE_SIZE = 32

    @staticmethod
    def get_knob_config():
        return {
            'epochs': IntegerKnob(1, 30),
            'learning_rate': FloatKnob(1e-3, 2e-1, is_exp=True),
            'momentum': FloatKnob(0.8, 0.95),
            'weight_decay': FloatKnob(1e-5, 1e-3, is_exp=True),
            'batch_size': CategoricalKnob([64, 128, 256]),
            'width_mult': CategoricalKnob([0.5, 1.0]),
            'image_size': FixedKnob(32),
        }

    def _engine_kwargs(self, num_classes, channels, image_size):
        k = self._knobs
        wm = float(k.get('width_mult', 1.0))
        cfg = tuple(v if v == 'M' else max(8, int(v * wm) // 8 * 8) for v in VGG_SMALL_CFG)
        return dict(cfg=cfg, fc_dims=(max(64, int(512 * wm)),), optimizer='sgd',
                    lr=float(k.get('learning_rate', 0.05)), momentum=float(k.get('momentum', 0.9)),
                    weight_decay=float(k.get('weight_decay', 5e-4)), nesterov=True)


class VggSmallTrial(VggSmall):
    """The benchmark's trial definition (bench.py phase 2): VggSmall at full width, batch 256, ten
    epochs over a CIFAR-sized train split (50k images), evaluated on 10k, parameters pickled — a
    full-dataset training run per trial, like the reference's TfVgg16 trials
    (examples/models/image_classification/TfVgg16.py:20-25).  The advisor searches the SGD knobs
    only, so every trial does the same work."""

    EPOCHS = 10

    @classmethod
    def get_knob_config(cls):
        return {
            'epochs': FixedKnob(cls.EPOCHS),
            'learning_rate': FloatKnob(1e-2, 2e-1, is_exp=True),
            'momentum': FloatKnob(0.8, 0.95),
            'weight_decay': FloatKnob(1e-5, 1e-3, is_exp=True),
            'batch_size': FixedKnob(256),
            'width_mult': FixedKnob(1.0),
            'image_size': FixedKnob(32),
        }



class VggSmallProbe(VggSmallTrial):
    """Overhead probe (bench.py phase 2b): the same trial at 2 epochs over 8192 images — about 64
    training steps, so per-trial fixed costs (claim, propose, build, capture, eval, dump) dominate."""

    EPOCHS = 2


if __name__ == '__main__':
    from rafiki_amd.model import test_model_class
    test_model_class(__file__, 'VggSmall', TaskType.IMAGE_CLASSIFICATION, {},
                     'synthetic://image?n=2048&size=32&channels=3&classes=10&seed=0',
                     'synthetic://image?n=512&size=32&channels=3&classes=10&seed=1',
                     knobs={'epochs': 2, 'learning_rate': 0.05, 'momentum': 0.9, 'weight_decay': 5e-4,
                            'batch_size': 128, 'width_mult': 0.5, 'image_size': 32})
