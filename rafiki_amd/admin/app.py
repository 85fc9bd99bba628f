"""Admin REST API (Flask) — same routes, roles and JSON shapes as the reference.

Reference parity: rafiki/admin/app.py:16-396 (route table in SURVEY §2.2).  CORS headers are set
manually (flask_cors is not available offline).  Uncaught errors return the traceback with HTTP
500 like the reference; authorization failures return 401/403.
"""
from __future__ import annotations

import traceback
from datetime import datetime

from flask import Flask, Response, jsonify, request

from ..constants import UserType
from ..utils.auth import UnauthorizedError, auth, generate_token
from .admin import Admin

_ADMIN = {'instance': None}


def set_admin(admin: Admin):
    _ADMIN['instance'] = admin


def get_admin() -> Admin:
    if _ADMIN['instance'] is None:
        _ADMIN['instance'] = Admin()
    return _ADMIN['instance']


def get_request_params():
    params = request.get_json(silent=True)
    if params is None:
        params = request.form.to_dict()
    params = dict(params or {})
    params.update({k: v for k, v in request.args.items()})
    return params


def create_app(admin: Admin = None) -> Flask:
    if admin is not None:
        set_admin(admin)
    app = Flask('rafiki_amd.admin')

    @app.after_request
    def cors(resp):
        resp.headers['Access-Control-Allow-Origin'] = '*'
        resp.headers['Access-Control-Allow-Headers'] = 'Authorization, Content-Type'
        resp.headers['Access-Control-Allow-Methods'] = 'GET, POST, DELETE, OPTIONS'
        return resp

    @app.errorhandler(UnauthorizedError)
    def unauthorized(e):
        return 'Unauthorized: {}'.format(e), 401

    @app.errorhandler(Exception)
    def handle_error(e):
        return traceback.format_exc(), 500

    @app.route('/')
    def index():
        return 'Rafiki Admin is up.'

    from ..utils.metrics import admin_gauges, instrument
    instrument(app, 'admin', admin_gauges(lambda: get_admin().db))

    # ------------------------------------------------------------------------------ users
    @app.route('/users', methods=['POST'])
    @auth([UserType.ADMIN])
    def create_user(a):
        p = get_request_params()
        if a['user_type'] != UserType.SUPERADMIN and p.get('user_type') in (UserType.ADMIN, UserType.SUPERADMIN):
            raise UnauthorizedError('only superadmins may create admins')
        return jsonify(get_admin().create_user(p['email'], p['password'], p['user_type']))

    @app.route('/users', methods=['GET'])
    @auth([UserType.ADMIN])
    def get_users(a):
        return jsonify(get_admin().get_users())

    @app.route('/users', methods=['DELETE'])
    @auth([UserType.ADMIN])
    def ban_user(a):
        p = get_request_params()
        adm = get_admin()
        user = adm.get_user_by_email(p['email'])
        if user is not None:
            if a['user_type'] != UserType.SUPERADMIN and user['user_type'] in (UserType.ADMIN, UserType.SUPERADMIN):
                raise UnauthorizedError('only superadmins may ban admins')
            if a['user_id'] == user['id']:
                raise UnauthorizedError('cannot ban yourself')
        return jsonify(adm.ban_user(p['email']))

    @app.route('/tokens', methods=['POST'])
    def generate_user_token():
        p = get_request_params()
        user = get_admin().authenticate_user(p['email'], p['password'])
        if user.get('banned_date') is not None and datetime.utcnow() > user['banned_date']:
            raise UnauthorizedError('User is banned')
        token = generate_token({'user_id': user['id'], 'user_type': user['user_type']})
        return jsonify({'user_id': user['id'], 'user_type': user['user_type'], 'token': token})

    # ------------------------------------------------------------------------- train jobs
    dev_roles = [UserType.ADMIN, UserType.MODEL_DEVELOPER, UserType.APP_DEVELOPER]

    @app.route('/train_jobs', methods=['POST'])
    @auth(dev_roles)
    def create_train_job(a):
        p = get_request_params()
        return jsonify(get_admin().create_train_job(a['user_id'], p['app'], p['task'], p['train_dataset_uri'],
                                                    p['test_dataset_uri'], p.get('budget') or {},
                                                    p.get('model_ids') or []))

    @app.route('/train_jobs', methods=['GET'])
    @auth(dev_roles)
    def get_train_jobs_by_user(a):
        p = get_request_params()
        uid = p.get('user_id', a['user_id'])
        if a['user_type'] not in (UserType.SUPERADMIN, UserType.ADMIN) and uid != a['user_id']:
            raise UnauthorizedError()
        return jsonify(get_admin().get_train_jobs_by_user(uid))

    @app.route('/train_jobs/<app_name>', methods=['GET'])
    @auth(dev_roles)
    def get_train_jobs_of_app(a, app_name):
        return jsonify(get_admin().get_train_jobs_by_app(a['user_id'], app_name))

    @app.route('/train_jobs/<app_name>/<app_version>', methods=['GET'])
    @auth(dev_roles)
    def get_train_job(a, app_name, app_version):
        return jsonify(get_admin().get_train_job(a['user_id'], app_name, int(app_version)))

    @app.route('/train_jobs/<app_name>/<app_version>/stop', methods=['POST'])
    @auth(dev_roles)
    def stop_train_job(a, app_name, app_version):
        return jsonify(get_admin().stop_train_job(a['user_id'], app_name, int(app_version)))

    @app.route('/train_jobs/<app_name>/<app_version>/trials', methods=['GET'])
    @auth(dev_roles)
    def get_trials_of_train_job(a, app_name, app_version):
        p = get_request_params()
        adm = get_admin()
        if p.get('type') == 'best':
            return jsonify(adm.get_best_trials_of_train_job(a['user_id'], app_name, int(app_version),
                                                            max_count=int(p.get('max_count', 2))))
        return jsonify(adm.get_trials_of_train_job(a['user_id'], app_name, int(app_version)))

    # ----------------------------------------------------------------------------- trials
    @app.route('/trials/<trial_id>/logs', methods=['GET'])
    @auth(dev_roles)
    def get_trial_logs(a, trial_id):
        return jsonify(get_admin().get_trial_logs(trial_id))

    @app.route('/trials/<trial_id>/parameters', methods=['GET'])
    @auth(dev_roles)
    def get_trial_parameters(a, trial_id):
        data = get_admin().get_trial_parameters(trial_id)
        return Response(data, mimetype='application/octet-stream')

    @app.route('/trials/<trial_id>', methods=['GET'])
    @auth(dev_roles)
    def get_trial(a, trial_id):
        return jsonify(get_admin().get_trial(trial_id))

    # --------------------------------------------------------------------- inference jobs
    @app.route('/inference_jobs', methods=['POST'])
    @auth(dev_roles)
    def create_inference_job(a):
        p = get_request_params()
        return jsonify(get_admin().create_inference_job(a['user_id'], p['app'], int(p.get('app_version', -1)),
                                                        max_models=p.get('max_models')))

    @app.route('/inference_jobs', methods=['GET'])
    @auth(dev_roles)
    def get_inference_jobs_by_user(a):
        p = get_request_params()
        uid = p.get('user_id', a['user_id'])
        if a['user_type'] not in (UserType.SUPERADMIN, UserType.ADMIN) and uid != a['user_id']:
            raise UnauthorizedError()
        return jsonify(get_admin().get_inference_jobs_by_user(uid))

    @app.route('/inference_jobs/<app_name>', methods=['GET'])
    @auth(dev_roles)
    def get_inference_jobs_of_app(a, app_name):
        return jsonify(get_admin().get_inference_jobs_of_app(a['user_id'], app_name))

    @app.route('/inference_jobs/<app_name>/<app_version>', methods=['GET'])
    @auth(dev_roles)
    def get_running_inference_job(a, app_name, app_version):
        return jsonify(get_admin().get_running_inference_job(a['user_id'], app_name, int(app_version)))

    @app.route('/inference_jobs/<app_name>/<app_version>/stop', methods=['POST'])
    @auth(dev_roles)
    def stop_inference_job(a, app_name, app_version):
        return jsonify(get_admin().stop_inference_job(a['user_id'], app_name, int(app_version)))

    # ----------------------------------------------------------------------------- models
    @app.route('/models', methods=['POST'])
    @auth([UserType.ADMIN, UserType.MODEL_DEVELOPER])
    def create_model(a):
        p = get_request_params()
        f = request.files.get('model_file_bytes')
        blob = f.read() if f is not None else p['model_file_bytes'].encode('utf-8')
        deps = p.get('dependencies') or {}
        if isinstance(deps, str):
            import json
            deps = json.loads(deps) if deps else {}
        return jsonify(get_admin().create_model(a['user_id'], p['name'], p['task'], blob, p['model_class'],
                                                p.get('docker_image'), deps, p.get('access_right') or 'PRIVATE'))

    @app.route('/models/available', methods=['GET'])
    @auth(dev_roles)
    def get_available_models(a):
        p = get_request_params()
        return jsonify(get_admin().get_available_models(a['user_id'], p.get('task')))

    @app.route('/models/<model_id>', methods=['GET'])
    @auth(dev_roles)
    def get_model(a, model_id):
        adm = get_admin()
        m = adm.get_model(model_id)
        if a['user_type'] not in (UserType.SUPERADMIN, UserType.ADMIN) and m['user_id'] != a['user_id']:
            raise UnauthorizedError()
        return jsonify(m)

    @app.route('/models/<model_id>', methods=['DELETE'])
    @auth([UserType.ADMIN, UserType.MODEL_DEVELOPER])
    def delete_model(a, model_id):
        adm = get_admin()
        m = adm.get_model(model_id)
        if a['user_type'] not in (UserType.SUPERADMIN, UserType.ADMIN) and m['user_id'] != a['user_id']:
            raise UnauthorizedError()
        return jsonify(adm.delete_model(model_id))

    @app.route('/models/<model_id>/model_file', methods=['GET'])
    @auth([UserType.ADMIN, UserType.MODEL_DEVELOPER])
    def download_model_file(a, model_id):
        adm = get_admin()
        m = adm.get_model(model_id)
        if a['user_type'] not in (UserType.SUPERADMIN, UserType.ADMIN) and m['user_id'] != a['user_id']:
            raise UnauthorizedError()
        return Response(adm.get_model_file(model_id), mimetype='application/octet-stream')

    # ----------------------------------------------------------------------------- admin
    @app.route('/actions/stop_all_jobs', methods=['POST'])
    @auth([])
    def stop_all_jobs(a):
        adm = get_admin()
        return jsonify({'train_jobs': adm.stop_all_train_jobs(), 'inference_jobs': adm.stop_all_inference_jobs()})

    @app.route('/event/<name>', methods=['POST'])
    @auth([])
    def handle_event(a, name):
        return jsonify(get_admin().handle_event(name, **get_request_params()))

    # --------------------------------------------------------------------------- web UI
    @app.route('/ui')
    @app.route('/ui/')
    def web_ui():
        from ..web import INDEX_HTML
        return Response(INDEX_HTML, mimetype='text/html')

    return app
