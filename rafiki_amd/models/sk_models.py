"""scikit-learn image classifiers (CPU): SkDt (decision tree) and SkSvm (SVC).

Reference: examples/models/image_classification/SkDt.py:12-84 (knobs max_depth Int(1,32),
criterion Cat(gini, entropy); params = base64 pickle) and SkSvm.py (max_iter Int(10,20), kernel
Cat(rbf, linear), gamma Cat(scale, auto), C Float(1e-2,1e2,exp)).  These are the BASELINE's
"SkDt ... on CPU (plumbing, no GPU)" config.  Parameters are pickled sklearn estimators produced
by this system's own workers (trusted), stored as base64 like the reference.
"""
import base64
import pickle

import numpy as np

from rafiki_amd.constants import TaskType  # noqa: F401
from rafiki_amd.model import BaseModel, CategoricalKnob, FloatKnob, IntegerKnob, dataset_utils, logger


class _SkImageModel(BaseModel):
    IMAGE_SIZE = 28

    def __init__(self, **knobs):
        super().__init__(**knobs)
        self._knobs = knobs
        self._clf = self._build()

    def _build(self):
        raise NotImplementedError

    def _xy(self, uri):
        ds = dataset_utils.load_dataset_of_image_files(uri, image_size=self.IMAGE_SIZE)
        images, labels = ds.as_arrays()
        return self._flat(images), np.asarray(labels)

    @staticmethod
    def _flat(images):
        x = np.asarray(images, dtype=np.float32)
        return x.reshape(x.shape[0], -1) / 255.0

    def train(self, dataset_uri):
        x, y = self._xy(dataset_uri)
        self._clf.fit(x, y)
        logger.log('Train accuracy: {}'.format(float((self._clf.predict(x) == y).mean())))

    def evaluate(self, dataset_uri):
        x, y = self._xy(dataset_uri)
        return float((self._clf.predict(x) == y).mean())

    def predict(self, queries):
        x = self._flat(dataset_utils.resize_as_images(queries, self.IMAGE_SIZE)
                       if np.asarray(queries[0]).shape[0] != self.IMAGE_SIZE else queries)
        probs = self._clf.predict_proba(x)
        # expand to the full class range so ensembles over models align
        full = np.zeros((len(queries), int(max(self._clf.classes_)) + 1))
        full[:, self._clf.classes_.astype(int)] = probs
        return full.tolist()

    def dump_parameters(self):
        return {'clf_base64': base64.b64encode(pickle.dumps(self._clf)).decode('utf-8')}

    def load_parameters(self, params):
        self._clf = pickle.loads(base64.b64decode(params['clf_base64'].encode('utf-8')))

    def destroy(self):
        pass


class SkDt(_SkImageModel):
    @staticmethod
    def get_knob_config():
        return {'max_depth': IntegerKnob(1, 32), 'criterion': CategoricalKnob(['gini', 'entropy'])}

    def _build(self):
        from sklearn.tree import DecisionTreeClassifier
        return DecisionTreeClassifier(max_depth=self._knobs.get('max_depth'), criterion=self._knobs.get('criterion',
                                                                                                         'gini'))


class SkSvm(_SkImageModel):
    @staticmethod
    def get_knob_config():
        return {'max_iter': IntegerKnob(10, 20), 'kernel': CategoricalKnob(['rbf', 'linear']),
                'gamma': CategoricalKnob(['scale', 'auto']), 'C': FloatKnob(1e-2, 1e2, is_exp=True)}

    def _build(self):
        from sklearn.svm import SVC
        return SVC(max_iter=self._knobs.get('max_iter', 20), kernel=self._knobs.get('kernel', 'rbf'),
                   gamma=self._knobs.get('gamma', 'scale'), C=self._knobs.get('C', 1.0), probability=True)
