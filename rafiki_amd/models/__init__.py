"""Model zoo: single-file BaseModel classes uploadable through the client.

  VggSmall (vgg_small.py)        gfx950 engine, the BASELINE benchmark architecture
  Vgg16 (vgg16.py)               gfx950 engine, TfVgg16 semantics (48x48x3, Adam)
  FeedForward (feed_forward.py)  gfx950 engine, TfFeedForward semantics
  SkDt, SkSvm (sk_models.py)     scikit-learn on CPU
  BigramHmm, PyBiLstm (pos_tagging.py)
  PgGan (pg_gan.py)              progressive GAN (image generation), data-parallel over RCCL
"""
import os

MODELS_DIR = os.path.dirname(os.path.abspath(__file__))
ZOO = {
    'VggSmall': ('vgg_small.py', 'IMAGE_CLASSIFICATION'),
    'VggSmallTrial': ('vgg_small.py', 'IMAGE_CLASSIFICATION'),
    'VggSmallProbe': ('vgg_small.py', 'IMAGE_CLASSIFICATION'),
    'Vgg16': ('vgg16.py', 'IMAGE_CLASSIFICATION'),
    'FeedForward': ('feed_forward.py', 'IMAGE_CLASSIFICATION'),
    'SkDt': ('sk_models.py', 'IMAGE_CLASSIFICATION'),
    'SkSvm': ('sk_models.py', 'IMAGE_CLASSIFICATION'),
    'BigramHmm': ('pos_tagging.py', 'POS_TAGGING'),
    'PyBiLstm': ('pos_tagging.py', 'POS_TAGGING'),
    'PgGan': ('pg_gan.py', 'IMAGE_GENERATION'),
}


def model_file(name):
    return os.path.join(MODELS_DIR, ZOO[name][0])
