"""Predictor HTTP service: ``POST /predict {"query": q} -> {"prediction": p}`` (reference
rafiki/predictor/app.py:23-30) plus ``POST /predict_batch {"queries": [...]}`` (the reference's
``predict_batch`` TODO, predictor.py:85-87).  Unauthenticated, like the reference.

Run as a service: ``python -m rafiki_amd.predictor.server`` with RAFIKI_INFERENCE_JOB_ID,
RAFIKI_SERVICE_ID and RAFIKI_SERVICE_PORT in the environment.  The service serves through the
native C++ front end (``nativeserve.NativePredictorServer``, same routes); RAFIKI_PREDICTOR_SERVER=fast
selects the asyncio one (``fastserve``) and RAFIKI_PREDICTOR_SERVER=flask this Flask app.
"""
from __future__ import annotations

import logging
import os
import sys
import traceback

from flask import Flask, Response, jsonify, request

logger = logging.getLogger(__name__)


def create_app(predictor):
    app = Flask('rafiki_amd.predictor')
    predictor.start()

    @app.errorhandler(Exception)
    def err(e):
        return traceback.format_exc(), 500

    @app.route('/')
    def index():
        return 'Rafiki Predictor is up.'

    from .. import runtime

    @app.route('/predict', methods=['POST'])
    def predict():
        raw = request.get_data(cache=True)
        arr = runtime.json_u8_array(raw, 'query')  # image queries: native parse, no per-pixel json
        if arr is not None:
            p = predictor.predict_one(arr)
        else:
            body = request.get_json(silent=True) or {}
            p = predictor.predict_one(body['query'])
        return jsonify({'prediction': p.tolist() if hasattr(p, 'tolist') else p})

    @app.route('/predict_batch', methods=['POST'])
    def predict_batch():
        raw = request.get_data(cache=True)
        arr = runtime.json_u8_array(raw, 'queries')
        if arr is not None:
            out = predictor.predict_array(arr)
            return jsonify({'predictions': out.tolist() if hasattr(out, 'tolist') else out})
        body = request.get_json(silent=True) or {}
        return jsonify({'predictions': predictor.predict(body['queries'])})

    @app.route('/predict_batch_npy', methods=['POST'])
    def predict_batch_npy():
        """Binary fast path: body = one ``.npy`` array (e.g. uint8 [Q, H, W(, C)] images), response =
        ``.npy`` float32 [Q, classes].  Skips JSON encode/decode of every pixel, which bounds the JSON
        endpoints at a few thousand images/s; the array goes straight to the device."""
        import io
        import numpy as np
        arr = np.load(io.BytesIO(request.get_data()), allow_pickle=False)
        probs = predictor.predict_array(arr)
        buf = io.BytesIO()
        np.save(buf, np.asarray(probs, dtype=np.float32), allow_pickle=False)
        return Response(buf.getvalue(), mimetype='application/octet-stream')

    from ..utils.metrics import instrument, predictor_gauges
    instrument(app, 'predictor', predictor_gauges(predictor))

    @app.route('/stats', methods=['GET'])
    def stats():
        return jsonify({**predictor.stats, 'models': [n for n, _ in predictor.models],
                        'resident_bytes': predictor.cache.used})

    return app


def main():
    from ..db.database import Database
    from ..utils.log import configure_logging
    from .predictor import Predictor
    sid = os.environ.get('RAFIKI_SERVICE_ID')
    configure_logging('service-{}-predictor'.format(sid))
    db = Database()
    try:
        predictor = Predictor.from_inference_job(os.environ['RAFIKI_INFERENCE_JOB_ID'], db=db)
    except Exception:
        logger.error(traceback.format_exc())
        if sid:
            db.mark_service_as_errored(db.get_service(sid))
        return 1
    port = int(os.environ.get('RAFIKI_SERVICE_PORT', '3003'))
    if os.environ.get('RAFIKI_PREDICTOR_SERVER', 'fast') == 'flask':
        app = create_app(predictor)
        if sid:
            db.mark_service_as_running(db.get_service(sid))
        app.run(host='0.0.0.0', port=port, threaded=True)
        return 0
    from .nativeserve import make_server
    srv = make_server(predictor, '0.0.0.0', port)
    if sid:
        db.mark_service_as_running(db.get_service(sid))
    srv.serve_forever()
    return 0


if __name__ == '__main__':
    sys.exit(main())
