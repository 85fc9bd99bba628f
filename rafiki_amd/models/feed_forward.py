"""FeedForward — TfFeedForward semantics on the gfx950 engine: Flatten -> BatchNorm -> (Dense+ReLU) x L
-> Dense -> softmax cross-entropy, Adam.

Reference: examples/models/image_classification/TfFeedForward.py:14-164 (knobs :20-28: epochs
Fixed 2, hidden_layer_count Int(1,2), hidden_layer_units Int(2,128),
learning_rate Float(1e-5,1e-1,exp), batch_size Cat(16..128), image_size Fixed 32).
"""
from rafiki_amd.constants import TaskType  # noqa: F401
from rafiki_amd.model import CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob
from rafiki_amd.models.image_classifier import NativeImageClassifier


class FeedForward(NativeImageClassifier):
    DEFAULT_IMAGE_SIZE = 32

    @staticmethod
    def get_knob_config():
        return {
            'epochs': FixedKnob(2),
            'hidden_layer_count': IntegerKnob(1, 2),
            'hidden_layer_units': IntegerKnob(2, 128),
            'learning_rate': FloatKnob(1e-5, 1e-1, is_exp=True),
            'batch_size': CategoricalKnob([16, 32, 64, 128]),
            'image_size': FixedKnob(32),
        }

    def _engine_kwargs(self, num_classes, channels, image_size):
        k = self._knobs
        units = int(k.get('hidden_layer_units', 64))
        layers = int(k.get('hidden_layer_count', 1))
        return dict(cfg=(), fc_dims=(units,) * layers, optimizer='adam', lr=float(k.get('learning_rate', 1e-3)),
                    weight_decay=0.0, input_bn=True, betas=(0.9, 0.999))

    def train(self, dataset_uri):
        self._knobs.setdefault('lr_schedule', 'constant')
        return super().train(dataset_uri)


if __name__ == '__main__':
    from rafiki_amd.model import test_model_class
    test_model_class(__file__, 'FeedForward', TaskType.IMAGE_CLASSIFICATION, {},
                     'synthetic://image?n=4096&size=28&channels=1&classes=10&seed=0',
                     'synthetic://image?n=1024&size=28&channels=1&classes=10&seed=1',
                     knobs={'epochs': 2, 'hidden_layer_count': 2, 'hidden_layer_units': 36, 'learning_rate': 0.01,
                            'batch_size': 32, 'image_size': 28})
