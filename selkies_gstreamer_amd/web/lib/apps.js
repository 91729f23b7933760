// Apps panel: a catalog of installable desktop apps (reference AppsModal,
// addons/selkies-dashboard/src/components/Sidebar.jsx:266-369: fetches an app
// metadata list, grid with search, install / remove / update through the server's
// command channel running proot-apps, installed names kept in localStorage).
// The catalog is JSON ({"apps": [{name, full_name, description, icon}]}) from the
// `apps_catalog_url` setting or ./apps.json next to the client.

export const INSTALLED_KEY = 'selkiesInstalledApps';
export const PROOT_APPS = '~/.local/bin/proot-apps';

// Normalised list of {name, title, description, icon}; entries without a
// shell-safe name are dropped (the name becomes part of a command line).
export function parseCatalog(data) {
  const list = Array.isArray(data) ? data : (data && Array.isArray(data.apps) ? data.apps : []);
  const out = [];
  for (const a of list) {
    if (!a || typeof a.name !== 'string' || !/^[A-Za-z0-9][A-Za-z0-9._+-]*$/.test(a.name)) continue;
    out.push({
      name: a.name,
      title: typeof a.full_name === 'string' && a.full_name ? a.full_name : a.name,
      description: typeof a.description === 'string' ? a.description : '',
      icon: typeof a.icon === 'string' ? a.icon : '',
    });
  }
  return out;
}

// Case-insensitive match on name, title and description.
export function filterApps(apps, term) {
  const q = String(term || '').trim().toLowerCase();
  if (!q) return apps.slice();
  return apps.filter((a) => a.name.toLowerCase().includes(q) || a.title.toLowerCase().includes(q)
    || a.description.toLowerCase().includes(q));
}

// Command-channel message for an action on an app ('cmd,' + a shell line the server
// runs when command_enabled; 'st' opens it in a terminal like the reference).
export function appCommand(action, name) {
  if (!['install', 'remove', 'update'].includes(action)) throw new Error(`unknown app action ${action}`);
  if (!/^[A-Za-z0-9][A-Za-z0-9._+-]*$/.test(name)) throw new Error(`unsafe app name ${name}`);
  return `cmd,st ${PROOT_APPS} ${action} ${name}`;
}

// Installed-app bookkeeping (a sorted, de-duplicated list of names).
export function loadInstalled(storage) {
  try {
    const v = JSON.parse((storage && storage.getItem(INSTALLED_KEY)) || '[]');
    return Array.isArray(v) ? [...new Set(v.filter((x) => typeof x === 'string'))].sort() : [];
  } catch (e) {
    return [];
  }
}

export function updateInstalled(list, action, name) {
  const s = new Set(list);
  if (action === 'install') s.add(name);
  if (action === 'remove') s.delete(name);
  return [...s].sort();
}

export function saveInstalled(storage, list) {
  if (storage) storage.setItem(INSTALLED_KEY, JSON.stringify(list));
}
