"""Two replicas behind the native front end (tests/test_serving_gpu.py two-replica test): for every answer
that differs from predict_array, which reference row does it match?  A row mix-up matches another image
exactly; a numeric difference matches none."""
import io
import json
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import requests
    from rafiki_amd.model.dataset import synthetic_images
    from rafiki_amd.models.vgg_small import VggSmall
    from rafiki_amd.parallel.context import TrialContext, use_context
    from rafiki_amd.predictor import nativeserve
    from rafiki_amd.predictor.predictor import Predictor
    TRAIN = 'synthetic://image?n=1024&size=32&channels=3&classes=10&seed=0'
    models = []
    with use_context(TrialContext(device=torch.device('cuda'))):
        for i in range(4):
            m = VggSmall(epochs=1, learning_rate=0.05, momentum=0.9, weight_decay=5e-4, batch_size=128,
                         width_mult=0.5, image_size=32, seed=i)
            m.train(TRAIN)
            models.append(('t%d' % i, m))

    def copy():
        out = []
        with use_context(TrialContext(device=torch.device('cuda'))):
            for name, m in models:
                c = type(m)(**m._knobs)
                c.load_parameters(m.dump_parameters())
                out.append((name, c))
        return out
    imgs, _ = synthetic_images(96, size=32, channels=3, classes=10, seed=9)
    ref = Predictor(models).predict_array(imgs)
    refc = Predictor(copy()).predict_array(imgs)
    print(json.dumps({'copy_vs_original': float(np.abs(ref - refc).max())}), flush=True)
    for trial in range(3):
        p = Predictor(copy(), replicas=[copy()])
        srv = nativeserve.NativePredictorServer(p, '127.0.0.1', 0).start()
        url = 'http://127.0.0.1:{}'.format(srv.port)
        out = []

        def npy_client(k):
            s = requests.Session()
            for j in range(3):
                lo = ((k * 3 + j) % 12) * 8
                buf = io.BytesIO()
                np.save(buf, imgs[lo:lo + 8], allow_pickle=False)
                r = s.post(url + '/predict_batch_npy', data=buf.getvalue())
                got = np.load(io.BytesIO(r.content), allow_pickle=False)
                for q in range(8):
                    out.append(('n', lo + q, got[q]))

        def json_client(k):
            s = requests.Session()
            for j in range(6):
                i = (k * 6 + j) % 96
                r = s.post(url + '/predict', json={'query': imgs[i].tolist()})
                out.append(('j', i, np.asarray(r.json()['prediction'], dtype=np.float32)))
        ts = [threading.Thread(target=npy_client, args=(k,)) for k in range(4)] + \
             [threading.Thread(target=json_client, args=(k,)) for k in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        srv.shutdown()
        bad = []
        for kind, i, got in out:
            d = float(np.abs(got - ref[i]).max())
            if d > 1e-5:
                dists = np.abs(ref - got[None]).max(1)
                j = int(dists.argmin())
                bad.append({'kind': kind, 'row': i, 'diff': d, 'closest_ref_row': j, 'closest_diff': float(dists[j])})
        print(json.dumps({'trial': trial, 'answers': len(out), 'bad': bad[:12], 'n_bad': len(bad),
                          'replays': [r.graphs.replays for r in p.replicas]}), flush=True)


if __name__ == '__main__':
    main()
