"""Model SDK: BaseModel, knobs, logger, dataset utils, local test harness."""
from .dataset import (CorpusDataset, ImageFilesDataset, ModelDatasetUtils, dataset_utils, synthetic_corpus,
                      synthetic_images, write_corpus_zip, write_image_files_zip)
from .knob import (BaseKnob, CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob, decode_knobs, deserialize_knob_config,
                   encode_knobs, serialize_knob_config)
from .log import LogType, ModelLogger, logger
from .model import (BaseModel, InvalidModelClassException, InvalidModelParamsException, load_model_class,
                    load_model_class_from_file, parse_model_install_command, test_model_class)

__all__ = [
    'BaseModel', 'BaseKnob', 'CategoricalKnob', 'FixedKnob', 'FloatKnob', 'IntegerKnob', 'serialize_knob_config',
    'deserialize_knob_config', 'encode_knobs', 'decode_knobs', 'ModelLogger', 'LogType', 'logger',
    'ModelDatasetUtils', 'dataset_utils', 'ImageFilesDataset', 'CorpusDataset', 'synthetic_images',
    'synthetic_corpus', 'write_image_files_zip', 'write_corpus_zip', 'test_model_class', 'load_model_class',
    'load_model_class_from_file', 'parse_model_install_command', 'InvalidModelClassException',
    'InvalidModelParamsException',
]
