"""Which batch sizes make the ensemble's predictions differ from the batch-96 ones (tests/test_serving_gpu
test_native_front_end_npy_and_two_replicas_double_buffered tolerance 1e-5)?  Prints per-bucket max
differences and the tuned configs of the grouped eval convs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from rafiki_amd.model.dataset import synthetic_images
    from rafiki_amd.models.vgg_small import VggSmall
    from rafiki_amd.ops import autotune
    from rafiki_amd.parallel.context import TrialContext, use_context
    from rafiki_amd.predictor.predictor import Predictor
    TRAIN = 'synthetic://image?n=1024&size=32&channels=3&classes=10&seed=0'
    models = []
    with use_context(TrialContext(device=torch.device('cuda'))):
        for i in range(4):
            m = VggSmall(epochs=1, learning_rate=0.05, momentum=0.9, weight_decay=5e-4, batch_size=128,
                         width_mult=0.5, image_size=32, seed=i)
            m.train(TRAIN)
            models.append(('t%d' % i, m))
    imgs, _ = synthetic_images(96, size=32, channels=3, classes=10, seed=9)
    p = Predictor(models)
    ref = p.predict_array(imgs)
    for n in (1, 8, 16, 32, 64, 96):
        for lo in (0, 8, 88):
            if lo + n > 96:
                continue
            got = p.predict_array(imgs[lo:lo + n])
            d = np.abs(got - ref[lo:lo + n])
            print(json.dumps({'n': n, 'lo': lo, 'max_diff': float(d.max()),
                              'rows_over_1e-5': int((d.max(1) > 1e-5).sum())}), flush=True)
    # per-model: the members' own predict vs the batch-96 one
    for name, m in models:
        a = np.asarray(m.predict([im.tolist() for im in imgs[:8]]))
        b = np.asarray(m.predict([im.tolist() for im in imgs]))[:8]
        print(json.dumps({'model': name, 'member_b8_vs_b96': float(np.abs(a - b).max())}), flush=True)
    keys = [k for k in autotune._cache if 'g' in str(k[0])[:3] or 'sf' in str(k[0])]
    for k in keys[:40]:
        print(json.dumps({'key': [str(x) for x in k], 'cfg': list(autotune._cache[k])}), flush=True)


if __name__ == '__main__':
    main()
