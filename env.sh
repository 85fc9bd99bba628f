# Deployment configuration (reference .env.sh:1-55), one MI355X node, no Docker/Swarm/Postgres/Redis:
# SQLite in the workdir, services are local processes (one per GPU group) started by the admin.
export APP_MODE=${APP_MODE:-DEV}
export WORKDIR_PATH=${WORKDIR_PATH:-$PWD/rafiki_workdir}
export DATA_DIR_PATH=${DATA_DIR_PATH:-data}
export LOGS_DIR_PATH=${LOGS_DIR_PATH:-logs}
export PARAMS_DIR_PATH=${PARAMS_DIR_PATH:-params}
export ADMIN_HOST=${ADMIN_HOST:-127.0.0.1}
export ADMIN_PORT=${ADMIN_PORT:-3000}
export ADVISOR_HOST=${ADVISOR_HOST:-127.0.0.1}
export ADVISOR_PORT=${ADVISOR_PORT:-3002}
export PREDICTOR_PORT=${PREDICTOR_PORT:-3003}
export APP_SECRET=${APP_SECRET:-rafiki}
export SUPERADMIN_PASSWORD=${SUPERADMIN_PASSWORD:-rafiki}
export RAFIKI_GPUS_PER_NODE=${RAFIKI_GPUS_PER_NODE:-8}
export RAFIKI_GRAD_BUCKET_MB=${RAFIKI_GRAD_BUCKET_MB:-32}
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
