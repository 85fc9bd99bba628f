"""Create users from a CSV (email,password,user_type) as superadmin (reference examples/scripts/seed_users.py)."""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from rafiki_amd.client import Client  # noqa: E402
from rafiki_amd.config import SUPERADMIN_EMAIL, SUPERADMIN_PASSWORD  # noqa: E402

if __name__ == '__main__':
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), 'users.csv')
    c = Client(admin_host=os.environ.get('ADMIN_HOST', '127.0.0.1'), admin_port=int(os.environ.get('ADMIN_PORT', 3000)))
    c.login(SUPERADMIN_EMAIL, SUPERADMIN_PASSWORD)
    with open(path) as f:
        for row in csv.DictReader(f):
            try:
                c.create_user(row['email'], row['password'], row['user_type'])
                print('created', row['email'])
            except Exception as e:
                print('skipped', row['email'], e)
