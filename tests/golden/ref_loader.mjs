// Node 12 ESM loader hook used ONLY by make_golden.py in the build
// container: /root/reference has no package.json, so its *.js files are
// forced to load as ES modules. Nothing here runs on the GPU box.
export async function getFormat(url, context, defaultGetFormat) {
  if (url.startsWith('file:///root/reference/') && url.endsWith('.js')) {
    return { format: 'module' };
  }
  return defaultGetFormat(url, context, defaultGetFormat);
}
