"""Advisor process entry: ``python -m rafiki_amd.advisor`` (reference scripts/start_advisor.py:1-10).
The reference runs Flask single-threaded because BTB's GP is not thread-safe; AdvisorService
serialises with a lock, so this server may be threaded."""
import sys


def main():
    from ..config import get_config
    from ..utils.log import configure_logging
    from .service import create_app
    configure_logging('advisor')
    create_app().run(host='0.0.0.0', port=get_config().advisor_port, threaded=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
