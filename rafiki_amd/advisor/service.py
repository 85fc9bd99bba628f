"""AdvisorService: in-memory advisors keyed by id + the advisor REST app.

Reference parity: rafiki/advisor/service.py:15-80 (create idempotent by id, propose, feedback
returning a new proposal, delete) and advisor/app.py:17-50 (routes, ADMIN/APP_DEV roles).  The
reference serves it single-threaded (``threaded=False``); here the service is thread-safe (each
advisor holds its own lock) so it can run threaded.  Extension: ``propose_batch``.
"""
from __future__ import annotations

import threading
import traceback
import uuid

from ..constants import AdvisorType, UserType
from ..model.knob import deserialize_knob_config
from .advisor import Advisor


class InvalidAdvisorError(Exception):
    pass


class AdvisorService:
    def __init__(self):
        self._advisors = {}
        self._lock = threading.Lock()

    def create_advisor(self, knob_config_str, advisor_id=None, advisor_type=AdvisorType.BTB_GP):
        with self._lock:
            if advisor_id is not None and advisor_id in self._advisors:
                return {'id': advisor_id, 'is_created': False}
            aid = advisor_id or str(uuid.uuid4())
            self._advisors[aid] = Advisor(deserialize_knob_config(knob_config_str), advisor_type)
            return {'id': aid, 'is_created': True}

    def delete_advisor(self, advisor_id):
        with self._lock:
            existed = self._advisors.pop(advisor_id, None) is not None
        return {'id': advisor_id, 'is_deleted': existed}

    def _get(self, advisor_id):
        a = self._advisors.get(advisor_id)
        if a is None:
            raise InvalidAdvisorError(advisor_id)
        return a

    def generate_proposal(self, advisor_id):
        return {'knobs': self._get(advisor_id).propose()}

    def generate_proposals(self, advisor_id, count):
        return {'knobs': self._get(advisor_id).propose_batch(int(count))}

    def feedback(self, advisor_id, knobs, score):
        a = self._get(advisor_id)
        a.feedback(knobs, score)
        return {'knobs': a.propose()}


def create_app(service: AdvisorService = None):
    from flask import Flask, jsonify, request

    from ..utils.auth import auth
    service = service or AdvisorService()
    app = Flask('rafiki_amd.advisor')
    roles = [UserType.ADMIN, UserType.APP_DEVELOPER]

    def params():
        p = request.get_json(silent=True)
        if p is None:
            p = request.form.to_dict()
        p = dict(p or {})
        p.update(request.args.items())
        return p

    @app.errorhandler(Exception)
    def err(e):
        return traceback.format_exc(), 500

    @app.route('/')
    def index():
        return 'Rafiki Advisor is up.'

    @app.route('/advisors', methods=['POST'])
    @auth(roles)
    def create_advisor(a):
        p = params()
        return jsonify(service.create_advisor(p['knob_config_str'], p.get('advisor_id'),
                                              p.get('advisor_type') or AdvisorType.BTB_GP))

    @app.route('/advisors/<advisor_id>/propose', methods=['POST'])
    @auth(roles)
    def propose(a, advisor_id):
        p = params()
        if 'count' in p:
            return jsonify(service.generate_proposals(advisor_id, p['count']))
        return jsonify(service.generate_proposal(advisor_id))

    @app.route('/advisors/<advisor_id>/feedback', methods=['POST'])
    @auth(roles)
    def feedback(a, advisor_id):
        p = params()
        return jsonify(service.feedback(advisor_id, p['knobs'], p['score']))

    @app.route('/advisors/<advisor_id>', methods=['DELETE'])
    @auth(roles)
    def delete(a, advisor_id):
        return jsonify(service.delete_advisor(advisor_id))

    return app
