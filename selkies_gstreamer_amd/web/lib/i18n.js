// Dashboard strings in the reference dashboard's 18 languages
// (addons/selkies-dashboard/src/translations.js: en es zh hi pt fr ru de tr it nl ar
// ko ja vi th fil da). Keys are this client's own (flat, dotted by panel); a
// missing key falls back to English, then to the key itself; `{name}` placeholders
// are filled from the vars object. pickLanguage(): ?lang= first, then the browser's
// preferred languages, then English.

const en = {
  'section.clipboard': 'Clipboard', 'section.stats': 'Stats',
  'menu.title': 'Menu',
  'section.video': 'Video',
  'section.audio': 'Audio',
  'section.screen': 'Resolution',
  'section.input': 'Input',
  'section.keys': 'Keys',
  'section.apps': 'Apps',
  'section.files': 'Files',
  'section.sharing': 'Sharing',
  'section.gamepads': 'Gamepads',
  'section.graphs': 'Graphs',
  'section.monitor': 'System monitor',
  'section.shortcuts': 'Shortcuts',
  'section.language': 'Language',
  'screen.manual': 'manual resolution',
  'screen.apply': 'apply',
  'screen.scaling': 'scaling',
  'screen.css': 'CSS scaling (no HiDPI)',
  'audio.bitrate': 'bitrate',
  'input.gaming': 'gaming mode (pointer lock)',
  'input.trackpad': 'trackpad mode',
  'input.keyboard': 'on-screen keyboard',
  'apps.search': 'search apps',
  'apps.install': 'install',
  'apps.remove': 'remove',
  'apps.update': 'update',
  'apps.run': 'run',
  'apps.command': 'command',
  'apps.empty': 'no apps found',
  'apps.error': 'could not load the app list',
  'files.open': 'open file browser',
  'files.close': 'close',
  'files.upload': 'upload',
  'sharing.viewOnly': 'view only',
  'sharing.player': 'player {n}',
  'sharing.copy': 'copy',
  'gamepads.touch': 'touch gamepad',
  'gamepads.none': 'no gamepads',
  'monitor.memory': 'memory',
  'shortcuts.menu': 'Menu',
  'shortcuts.fullscreen': 'Fullscreen',
  'shortcuts.pointer': 'Pointer lock',
};

const es = {
  'section.clipboard': 'Portapapeles', 'section.stats': 'Estadísticas',
  'menu.title': 'Menú', 'section.video': 'Vídeo', 'section.audio': 'Audio', 'section.screen': 'Resolución',
  'section.input': 'Entrada', 'section.keys': 'Teclas', 'section.apps': 'Aplicaciones', 'section.files': 'Archivos',
  'section.sharing': 'Compartir', 'section.gamepads': 'Mandos', 'section.graphs': 'Gráficas',
  'section.monitor': 'Monitor del sistema', 'section.shortcuts': 'Atajos', 'section.language': 'Idioma',
  'screen.manual': 'resolución manual', 'screen.apply': 'aplicar', 'screen.scaling': 'escala',
  'screen.css': 'escala CSS (sin HiDPI)', 'audio.bitrate': 'tasa de bits',
  'input.gaming': 'modo juego (bloqueo del puntero)', 'input.trackpad': 'modo panel táctil',
  'input.keyboard': 'teclado en pantalla', 'apps.search': 'buscar aplicaciones', 'apps.install': 'instalar',
  'apps.remove': 'quitar', 'apps.update': 'actualizar', 'apps.run': 'ejecutar', 'apps.command': 'comando',
  'apps.empty': 'no se encontraron aplicaciones', 'apps.error': 'no se pudo cargar la lista de aplicaciones',
  'files.open': 'abrir el explorador de archivos', 'files.close': 'cerrar', 'files.upload': 'subir',
  'sharing.viewOnly': 'solo ver', 'sharing.player': 'jugador {n}', 'sharing.copy': 'copiar',
  'gamepads.touch': 'mando táctil', 'gamepads.none': 'sin mandos', 'monitor.memory': 'memoria',
  'shortcuts.menu': 'Menú', 'shortcuts.fullscreen': 'Pantalla completa', 'shortcuts.pointer': 'Bloquear puntero',
};

const zh = {
  'section.clipboard': '剪贴板', 'section.stats': '统计',
  'menu.title': '菜单', 'section.video': '视频', 'section.audio': '音频', 'section.screen': '分辨率',
  'section.input': '输入', 'section.keys': '按键', 'section.apps': '应用', 'section.files': '文件',
  'section.sharing': '共享', 'section.gamepads': '游戏手柄', 'section.graphs': '图表',
  'section.monitor': '系统监视器', 'section.shortcuts': '快捷键', 'section.language': '语言',
  'screen.manual': '手动分辨率', 'screen.apply': '应用', 'screen.scaling': '缩放',
  'screen.css': 'CSS 缩放（无 HiDPI）', 'audio.bitrate': '码率', 'input.gaming': '游戏模式（锁定指针）',
  'input.trackpad': '触控板模式', 'input.keyboard': '屏幕键盘', 'apps.search': '搜索应用', 'apps.install': '安装',
  'apps.remove': '移除', 'apps.update': '更新', 'apps.run': '运行', 'apps.command': '命令',
  'apps.empty': '未找到应用', 'apps.error': '无法加载应用列表', 'files.open': '打开文件浏览器',
  'files.close': '关闭', 'files.upload': '上传', 'sharing.viewOnly': '仅观看', 'sharing.player': '玩家 {n}',
  'sharing.copy': '复制', 'gamepads.touch': '触屏手柄', 'gamepads.none': '没有游戏手柄', 'monitor.memory': '内存',
  'shortcuts.menu': '菜单', 'shortcuts.fullscreen': '全屏', 'shortcuts.pointer': '锁定指针',
};

const hi = {
  'section.clipboard': 'क्लिपबोर्ड', 'section.stats': 'आँकड़े',
  'menu.title': 'मेनू', 'section.video': 'वीडियो', 'section.audio': 'ऑडियो', 'section.screen': 'रिज़ॉल्यूशन',
  'section.input': 'इनपुट', 'section.keys': 'कुंजियाँ', 'section.apps': 'ऐप्स', 'section.files': 'फ़ाइलें',
  'section.sharing': 'साझा करना', 'section.gamepads': 'गेमपैड', 'section.graphs': 'ग्राफ़',
  'section.monitor': 'सिस्टम मॉनिटर', 'section.shortcuts': 'शॉर्टकट', 'section.language': 'भाषा',
  'screen.manual': 'मैनुअल रिज़ॉल्यूशन', 'screen.apply': 'लागू करें', 'screen.scaling': 'स्केलिंग',
  'screen.css': 'CSS स्केलिंग (HiDPI नहीं)', 'audio.bitrate': 'बिटरेट', 'input.gaming': 'गेमिंग मोड (पॉइंटर लॉक)',
  'input.trackpad': 'ट्रैकपैड मोड', 'input.keyboard': 'ऑन-स्क्रीन कीबोर्ड', 'apps.search': 'ऐप्स खोजें',
  'apps.install': 'इंस्टॉल करें', 'apps.remove': 'हटाएँ', 'apps.update': 'अपडेट करें', 'apps.run': 'चलाएँ',
  'apps.command': 'कमांड', 'apps.empty': 'कोई ऐप नहीं मिला', 'apps.error': 'ऐप सूची लोड नहीं हो सकी',
  'files.open': 'फ़ाइल ब्राउज़र खोलें', 'files.close': 'बंद करें', 'files.upload': 'अपलोड करें',
  'sharing.viewOnly': 'केवल देखें', 'sharing.player': 'खिलाड़ी {n}', 'sharing.copy': 'कॉपी करें',
  'gamepads.touch': 'टच गेमपैड', 'gamepads.none': 'कोई गेमपैड नहीं', 'monitor.memory': 'मेमोरी',
  'shortcuts.menu': 'मेनू', 'shortcuts.fullscreen': 'पूर्ण स्क्रीन', 'shortcuts.pointer': 'पॉइंटर लॉक',
};

const pt = {
  'section.clipboard': 'Área de transferência', 'section.stats': 'Estatísticas',
  'menu.title': 'Menu', 'section.video': 'Vídeo', 'section.audio': 'Áudio', 'section.screen': 'Resolução',
  'section.input': 'Entrada', 'section.keys': 'Teclas', 'section.apps': 'Aplicativos', 'section.files': 'Arquivos',
  'section.sharing': 'Compartilhar', 'section.gamepads': 'Controles', 'section.graphs': 'Gráficos',
  'section.monitor': 'Monitor do sistema', 'section.shortcuts': 'Atalhos', 'section.language': 'Idioma',
  'screen.manual': 'resolução manual', 'screen.apply': 'aplicar', 'screen.scaling': 'escala',
  'screen.css': 'escala CSS (sem HiDPI)', 'audio.bitrate': 'taxa de bits',
  'input.gaming': 'modo jogo (travar ponteiro)', 'input.trackpad': 'modo trackpad', 'input.keyboard': 'teclado na tela',
  'apps.search': 'procurar aplicativos', 'apps.install': 'instalar', 'apps.remove': 'remover',
  'apps.update': 'atualizar', 'apps.run': 'executar', 'apps.command': 'comando',
  'apps.empty': 'nenhum aplicativo encontrado', 'apps.error': 'não foi possível carregar a lista de aplicativos',
  'files.open': 'abrir o navegador de arquivos', 'files.close': 'fechar', 'files.upload': 'enviar',
  'sharing.viewOnly': 'somente visualizar', 'sharing.player': 'jogador {n}', 'sharing.copy': 'copiar',
  'gamepads.touch': 'controle na tela', 'gamepads.none': 'nenhum controle', 'monitor.memory': 'memória',
  'shortcuts.menu': 'Menu', 'shortcuts.fullscreen': 'Tela cheia', 'shortcuts.pointer': 'Travar ponteiro',
};

const fr = {
  'section.clipboard': 'Presse-papiers', 'section.stats': 'Statistiques',
  'menu.title': 'Menu', 'section.video': 'Vidéo', 'section.audio': 'Audio', 'section.screen': 'Résolution',
  'section.input': 'Saisie', 'section.keys': 'Touches', 'section.apps': 'Applications', 'section.files': 'Fichiers',
  'section.sharing': 'Partage', 'section.gamepads': 'Manettes', 'section.graphs': 'Graphiques',
  'section.monitor': 'Moniteur système', 'section.shortcuts': 'Raccourcis', 'section.language': 'Langue',
  'screen.manual': 'résolution manuelle', 'screen.apply': 'appliquer', 'screen.scaling': 'mise à l\'échelle',
  'screen.css': 'mise à l\'échelle CSS (sans HiDPI)', 'audio.bitrate': 'débit',
  'input.gaming': 'mode jeu (verrouillage du pointeur)', 'input.trackpad': 'mode pavé tactile',
  'input.keyboard': 'clavier à l\'écran', 'apps.search': 'rechercher des applications', 'apps.install': 'installer',
  'apps.remove': 'supprimer', 'apps.update': 'mettre à jour', 'apps.run': 'lancer', 'apps.command': 'commande',
  'apps.empty': 'aucune application trouvée', 'apps.error': 'impossible de charger la liste des applications',
  'files.open': 'ouvrir l\'explorateur de fichiers', 'files.close': 'fermer', 'files.upload': 'téléverser',
  'sharing.viewOnly': 'lecture seule', 'sharing.player': 'joueur {n}', 'sharing.copy': 'copier',
  'gamepads.touch': 'manette tactile', 'gamepads.none': 'aucune manette', 'monitor.memory': 'mémoire',
  'shortcuts.menu': 'Menu', 'shortcuts.fullscreen': 'Plein écran', 'shortcuts.pointer': 'Verrouiller le pointeur',
};

const ru = {
  'section.clipboard': 'Буфер обмена', 'section.stats': 'Статистика',
  'menu.title': 'Меню', 'section.video': 'Видео', 'section.audio': 'Звук', 'section.screen': 'Разрешение',
  'section.input': 'Ввод', 'section.keys': 'Клавиши', 'section.apps': 'Приложения', 'section.files': 'Файлы',
  'section.sharing': 'Общий доступ', 'section.gamepads': 'Геймпады', 'section.graphs': 'Графики',
  'section.monitor': 'Системный монитор', 'section.shortcuts': 'Сочетания клавиш', 'section.language': 'Язык',
  'screen.manual': 'ручное разрешение', 'screen.apply': 'применить', 'screen.scaling': 'масштаб',
  'screen.css': 'масштаб CSS (без HiDPI)', 'audio.bitrate': 'битрейт',
  'input.gaming': 'игровой режим (захват указателя)', 'input.trackpad': 'режим тачпада',
  'input.keyboard': 'экранная клавиатура', 'apps.search': 'поиск приложений', 'apps.install': 'установить',
  'apps.remove': 'удалить', 'apps.update': 'обновить', 'apps.run': 'запустить', 'apps.command': 'команда',
  'apps.empty': 'приложения не найдены', 'apps.error': 'не удалось загрузить список приложений',
  'files.open': 'открыть файловый менеджер', 'files.close': 'закрыть', 'files.upload': 'загрузить',
  'sharing.viewOnly': 'только просмотр', 'sharing.player': 'игрок {n}', 'sharing.copy': 'копировать',
  'gamepads.touch': 'сенсорный геймпад', 'gamepads.none': 'нет геймпадов', 'monitor.memory': 'память',
  'shortcuts.menu': 'Меню', 'shortcuts.fullscreen': 'Полный экран', 'shortcuts.pointer': 'Захват указателя',
};

const de = {
  'section.clipboard': 'Zwischenablage', 'section.stats': 'Statistik',
  'menu.title': 'Menü', 'section.video': 'Video', 'section.audio': 'Audio', 'section.screen': 'Auflösung',
  'section.input': 'Eingabe', 'section.keys': 'Tasten', 'section.apps': 'Apps', 'section.files': 'Dateien',
  'section.sharing': 'Teilen', 'section.gamepads': 'Gamepads', 'section.graphs': 'Diagramme',
  'section.monitor': 'Systemmonitor', 'section.shortcuts': 'Tastenkürzel', 'section.language': 'Sprache',
  'screen.manual': 'manuelle Auflösung', 'screen.apply': 'übernehmen', 'screen.scaling': 'Skalierung',
  'screen.css': 'CSS-Skalierung (kein HiDPI)', 'audio.bitrate': 'Bitrate',
  'input.gaming': 'Spielmodus (Zeigersperre)', 'input.trackpad': 'Trackpad-Modus',
  'input.keyboard': 'Bildschirmtastatur', 'apps.search': 'Apps suchen', 'apps.install': 'installieren',
  'apps.remove': 'entfernen', 'apps.update': 'aktualisieren', 'apps.run': 'ausführen', 'apps.command': 'Befehl',
  'apps.empty': 'keine Apps gefunden', 'apps.error': 'App-Liste konnte nicht geladen werden',
  'files.open': 'Dateibrowser öffnen', 'files.close': 'schließen', 'files.upload': 'hochladen',
  'sharing.viewOnly': 'nur ansehen', 'sharing.player': 'Spieler {n}', 'sharing.copy': 'kopieren',
  'gamepads.touch': 'Touch-Gamepad', 'gamepads.none': 'keine Gamepads', 'monitor.memory': 'Speicher',
  'shortcuts.menu': 'Menü', 'shortcuts.fullscreen': 'Vollbild', 'shortcuts.pointer': 'Zeigersperre',
};

const tr = {
  'section.clipboard': 'Pano', 'section.stats': 'İstatistikler',
  'menu.title': 'Menü', 'section.video': 'Video', 'section.audio': 'Ses', 'section.screen': 'Çözünürlük',
  'section.input': 'Giriş', 'section.keys': 'Tuşlar', 'section.apps': 'Uygulamalar', 'section.files': 'Dosyalar',
  'section.sharing': 'Paylaşım', 'section.gamepads': 'Oyun kumandaları', 'section.graphs': 'Grafikler',
  'section.monitor': 'Sistem izleyici', 'section.shortcuts': 'Kısayollar', 'section.language': 'Dil',
  'screen.manual': 'elle çözünürlük', 'screen.apply': 'uygula', 'screen.scaling': 'ölçekleme',
  'screen.css': 'CSS ölçekleme (HiDPI yok)', 'audio.bitrate': 'bit hızı',
  'input.gaming': 'oyun modu (işaretçi kilidi)', 'input.trackpad': 'dokunmatik yüzey modu',
  'input.keyboard': 'ekran klavyesi', 'apps.search': 'uygulama ara', 'apps.install': 'yükle', 'apps.remove': 'kaldır',
  'apps.update': 'güncelle', 'apps.run': 'çalıştır', 'apps.command': 'komut', 'apps.empty': 'uygulama bulunamadı',
  'apps.error': 'uygulama listesi yüklenemedi', 'files.open': 'dosya tarayıcısını aç', 'files.close': 'kapat',
  'files.upload': 'yükle', 'sharing.viewOnly': 'yalnızca izle', 'sharing.player': 'oyuncu {n}',
  'sharing.copy': 'kopyala', 'gamepads.touch': 'dokunmatik kumanda', 'gamepads.none': 'kumanda yok',
  'monitor.memory': 'bellek', 'shortcuts.menu': 'Menü', 'shortcuts.fullscreen': 'Tam ekran',
  'shortcuts.pointer': 'İşaretçi kilidi',
};

const it = {
  'section.clipboard': 'Appunti', 'section.stats': 'Statistiche',
  'menu.title': 'Menu', 'section.video': 'Video', 'section.audio': 'Audio', 'section.screen': 'Risoluzione',
  'section.input': 'Input', 'section.keys': 'Tasti', 'section.apps': 'App', 'section.files': 'File',
  'section.sharing': 'Condivisione', 'section.gamepads': 'Gamepad', 'section.graphs': 'Grafici',
  'section.monitor': 'Monitor di sistema', 'section.shortcuts': 'Scorciatoie', 'section.language': 'Lingua',
  'screen.manual': 'risoluzione manuale', 'screen.apply': 'applica', 'screen.scaling': 'scala',
  'screen.css': 'scala CSS (senza HiDPI)', 'audio.bitrate': 'bitrate',
  'input.gaming': 'modalità gioco (blocco puntatore)', 'input.trackpad': 'modalità trackpad',
  'input.keyboard': 'tastiera su schermo', 'apps.search': 'cerca app', 'apps.install': 'installa',
  'apps.remove': 'rimuovi', 'apps.update': 'aggiorna', 'apps.run': 'esegui', 'apps.command': 'comando',
  'apps.empty': 'nessuna app trovata', 'apps.error': 'impossibile caricare l\'elenco delle app',
  'files.open': 'apri il browser dei file', 'files.close': 'chiudi', 'files.upload': 'carica',
  'sharing.viewOnly': 'solo visione', 'sharing.player': 'giocatore {n}', 'sharing.copy': 'copia',
  'gamepads.touch': 'gamepad touch', 'gamepads.none': 'nessun gamepad', 'monitor.memory': 'memoria',
  'shortcuts.menu': 'Menu', 'shortcuts.fullscreen': 'Schermo intero', 'shortcuts.pointer': 'Blocco puntatore',
};

const nl = {
  'section.clipboard': 'Klembord', 'section.stats': 'Statistieken',
  'menu.title': 'Menu', 'section.video': 'Video', 'section.audio': 'Audio', 'section.screen': 'Resolutie',
  'section.input': 'Invoer', 'section.keys': 'Toetsen', 'section.apps': 'Apps', 'section.files': 'Bestanden',
  'section.sharing': 'Delen', 'section.gamepads': 'Gamepads', 'section.graphs': 'Grafieken',
  'section.monitor': 'Systeemmonitor', 'section.shortcuts': 'Sneltoetsen', 'section.language': 'Taal',
  'screen.manual': 'handmatige resolutie', 'screen.apply': 'toepassen', 'screen.scaling': 'schaal',
  'screen.css': 'CSS-schaal (geen HiDPI)', 'audio.bitrate': 'bitrate',
  'input.gaming': 'gamemodus (aanwijzer vergrendelen)', 'input.trackpad': 'trackpadmodus',
  'input.keyboard': 'schermtoetsenbord', 'apps.search': 'apps zoeken', 'apps.install': 'installeren',
  'apps.remove': 'verwijderen', 'apps.update': 'bijwerken', 'apps.run': 'uitvoeren', 'apps.command': 'opdracht',
  'apps.empty': 'geen apps gevonden', 'apps.error': 'de lijst met apps kon niet worden geladen',
  'files.open': 'bestandsbrowser openen', 'files.close': 'sluiten', 'files.upload': 'uploaden',
  'sharing.viewOnly': 'alleen kijken', 'sharing.player': 'speler {n}', 'sharing.copy': 'kopiëren',
  'gamepads.touch': 'aanraakgamepad', 'gamepads.none': 'geen gamepads', 'monitor.memory': 'geheugen',
  'shortcuts.menu': 'Menu', 'shortcuts.fullscreen': 'Volledig scherm', 'shortcuts.pointer': 'Aanwijzer vergrendelen',
};

const ar = {
  'section.clipboard': 'الحافظة', 'section.stats': 'الإحصائيات',
  'menu.title': 'القائمة', 'section.video': 'الفيديو', 'section.audio': 'الصوت', 'section.screen': 'الدقة',
  'section.input': 'الإدخال', 'section.keys': 'المفاتيح', 'section.apps': 'التطبيقات', 'section.files': 'الملفات',
  'section.sharing': 'المشاركة', 'section.gamepads': 'أذرع التحكم', 'section.graphs': 'الرسوم البيانية',
  'section.monitor': 'مراقب النظام', 'section.shortcuts': 'الاختصارات', 'section.language': 'اللغة',
  'screen.manual': 'دقة يدوية', 'screen.apply': 'تطبيق', 'screen.scaling': 'التحجيم',
  'screen.css': 'تحجيم CSS (بدون HiDPI)', 'audio.bitrate': 'معدل البت', 'input.gaming': 'وضع الألعاب (قفل المؤشر)',
  'input.trackpad': 'وضع لوحة اللمس', 'input.keyboard': 'لوحة المفاتيح على الشاشة', 'apps.search': 'البحث عن تطبيقات',
  'apps.install': 'تثبيت', 'apps.remove': 'إزالة', 'apps.update': 'تحديث', 'apps.run': 'تشغيل', 'apps.command': 'أمر',
  'apps.empty': 'لم يتم العثور على تطبيقات', 'apps.error': 'تعذر تحميل قائمة التطبيقات',
  'files.open': 'فتح مستعرض الملفات', 'files.close': 'إغلاق', 'files.upload': 'رفع', 'sharing.viewOnly': 'مشاهدة فقط',
  'sharing.player': 'اللاعب {n}', 'sharing.copy': 'نسخ', 'gamepads.touch': 'ذراع تحكم باللمس',
  'gamepads.none': 'لا توجد أذرع تحكم', 'monitor.memory': 'الذاكرة', 'shortcuts.menu': 'القائمة',
  'shortcuts.fullscreen': 'ملء الشاشة', 'shortcuts.pointer': 'قفل المؤشر',
};

const ko = {
  'section.clipboard': '클립보드', 'section.stats': '통계',
  'menu.title': '메뉴', 'section.video': '비디오', 'section.audio': '오디오', 'section.screen': '해상도',
  'section.input': '입력', 'section.keys': '키', 'section.apps': '앱', 'section.files': '파일', 'section.sharing': '공유',
  'section.gamepads': '게임패드', 'section.graphs': '그래프', 'section.monitor': '시스템 모니터',
  'section.shortcuts': '단축키', 'section.language': '언어', 'screen.manual': '수동 해상도', 'screen.apply': '적용',
  'screen.scaling': '배율', 'screen.css': 'CSS 배율 (HiDPI 없음)', 'audio.bitrate': '비트레이트',
  'input.gaming': '게임 모드 (포인터 잠금)', 'input.trackpad': '트랙패드 모드', 'input.keyboard': '화면 키보드',
  'apps.search': '앱 검색', 'apps.install': '설치', 'apps.remove': '제거', 'apps.update': '업데이트', 'apps.run': '실행',
  'apps.command': '명령', 'apps.empty': '앱을 찾을 수 없습니다', 'apps.error': '앱 목록을 불러올 수 없습니다',
  'files.open': '파일 브라우저 열기', 'files.close': '닫기', 'files.upload': '업로드', 'sharing.viewOnly': '보기 전용',
  'sharing.player': '플레이어 {n}', 'sharing.copy': '복사', 'gamepads.touch': '터치 게임패드',
  'gamepads.none': '게임패드 없음', 'monitor.memory': '메모리', 'shortcuts.menu': '메뉴', 'shortcuts.fullscreen': '전체 화면',
  'shortcuts.pointer': '포인터 잠금',
};

const ja = {
  'section.clipboard': 'クリップボード', 'section.stats': '統計',
  'menu.title': 'メニュー', 'section.video': 'ビデオ', 'section.audio': 'オーディオ', 'section.screen': '解像度',
  'section.input': '入力', 'section.keys': 'キー', 'section.apps': 'アプリ', 'section.files': 'ファイル',
  'section.sharing': '共有', 'section.gamepads': 'ゲームパッド', 'section.graphs': 'グラフ',
  'section.monitor': 'システムモニター', 'section.shortcuts': 'ショートカット', 'section.language': '言語',
  'screen.manual': '手動解像度', 'screen.apply': '適用', 'screen.scaling': '拡大率', 'screen.css': 'CSS 拡大（HiDPI なし）',
  'audio.bitrate': 'ビットレート', 'input.gaming': 'ゲームモード（ポインターロック）', 'input.trackpad': 'トラックパッドモード',
  'input.keyboard': 'スクリーンキーボード', 'apps.search': 'アプリを検索', 'apps.install': 'インストール',
  'apps.remove': '削除', 'apps.update': '更新', 'apps.run': '実行', 'apps.command': 'コマンド',
  'apps.empty': 'アプリが見つかりません', 'apps.error': 'アプリ一覧を読み込めませんでした',
  'files.open': 'ファイルブラウザーを開く', 'files.close': '閉じる', 'files.upload': 'アップロード',
  'sharing.viewOnly': '閲覧のみ', 'sharing.player': 'プレイヤー {n}', 'sharing.copy': 'コピー',
  'gamepads.touch': 'タッチゲームパッド', 'gamepads.none': 'ゲームパッドなし', 'monitor.memory': 'メモリ',
  'shortcuts.menu': 'メニュー', 'shortcuts.fullscreen': '全画面', 'shortcuts.pointer': 'ポインターロック',
};

const vi = {
  'section.clipboard': 'Bộ nhớ tạm', 'section.stats': 'Thống kê',
  'menu.title': 'Menu', 'section.video': 'Video', 'section.audio': 'Âm thanh', 'section.screen': 'Độ phân giải',
  'section.input': 'Nhập liệu', 'section.keys': 'Phím', 'section.apps': 'Ứng dụng', 'section.files': 'Tệp',
  'section.sharing': 'Chia sẻ', 'section.gamepads': 'Tay cầm', 'section.graphs': 'Biểu đồ',
  'section.monitor': 'Giám sát hệ thống', 'section.shortcuts': 'Phím tắt', 'section.language': 'Ngôn ngữ',
  'screen.manual': 'độ phân giải thủ công', 'screen.apply': 'áp dụng', 'screen.scaling': 'tỉ lệ',
  'screen.css': 'tỉ lệ CSS (không HiDPI)', 'audio.bitrate': 'tốc độ bit', 'input.gaming': 'chế độ chơi game (khóa con trỏ)',
  'input.trackpad': 'chế độ bàn di chuột', 'input.keyboard': 'bàn phím ảo', 'apps.search': 'tìm ứng dụng',
  'apps.install': 'cài đặt', 'apps.remove': 'gỡ bỏ', 'apps.update': 'cập nhật', 'apps.run': 'chạy', 'apps.command': 'lệnh',
  'apps.empty': 'không tìm thấy ứng dụng', 'apps.error': 'không tải được danh sách ứng dụng',
  'files.open': 'mở trình duyệt tệp', 'files.close': 'đóng', 'files.upload': 'tải lên', 'sharing.viewOnly': 'chỉ xem',
  'sharing.player': 'người chơi {n}', 'sharing.copy': 'sao chép', 'gamepads.touch': 'tay cầm cảm ứng',
  'gamepads.none': 'không có tay cầm', 'monitor.memory': 'bộ nhớ', 'shortcuts.menu': 'Menu',
  'shortcuts.fullscreen': 'Toàn màn hình', 'shortcuts.pointer': 'Khóa con trỏ',
};

const th = {
  'section.clipboard': 'คลิปบอร์ด', 'section.stats': 'สถิติ',
  'menu.title': 'เมนู', 'section.video': 'วิดีโอ', 'section.audio': 'เสียง', 'section.screen': 'ความละเอียด',
  'section.input': 'อินพุต', 'section.keys': 'ปุ่ม', 'section.apps': 'แอป', 'section.files': 'ไฟล์',
  'section.sharing': 'การแชร์', 'section.gamepads': 'จอยเกม', 'section.graphs': 'กราฟ',
  'section.monitor': 'ตัวตรวจสอบระบบ', 'section.shortcuts': 'ปุ่มลัด', 'section.language': 'ภาษา',
  'screen.manual': 'กำหนดความละเอียดเอง', 'screen.apply': 'ใช้', 'screen.scaling': 'การปรับขนาด',
  'screen.css': 'ปรับขนาดด้วย CSS (ไม่มี HiDPI)', 'audio.bitrate': 'บิตเรต', 'input.gaming': 'โหมดเกม (ล็อกตัวชี้)',
  'input.trackpad': 'โหมดแทร็กแพด', 'input.keyboard': 'แป้นพิมพ์บนหน้าจอ', 'apps.search': 'ค้นหาแอป',
  'apps.install': 'ติดตั้ง', 'apps.remove': 'ลบ', 'apps.update': 'อัปเดต', 'apps.run': 'เรียกใช้', 'apps.command': 'คำสั่ง',
  'apps.empty': 'ไม่พบแอป', 'apps.error': 'โหลดรายการแอปไม่ได้', 'files.open': 'เปิดตัวเรียกดูไฟล์',
  'files.close': 'ปิด', 'files.upload': 'อัปโหลด', 'sharing.viewOnly': 'ดูอย่างเดียว', 'sharing.player': 'ผู้เล่น {n}',
  'sharing.copy': 'คัดลอก', 'gamepads.touch': 'จอยเกมแบบสัมผัส', 'gamepads.none': 'ไม่มีจอยเกม',
  'monitor.memory': 'หน่วยความจำ', 'shortcuts.menu': 'เมนู', 'shortcuts.fullscreen': 'เต็มหน้าจอ',
  'shortcuts.pointer': 'ล็อกตัวชี้',
};

const fil = {
  'section.clipboard': 'Clipboard', 'section.stats': 'Mga istatistika',
  'menu.title': 'Menu', 'section.video': 'Video', 'section.audio': 'Audio', 'section.screen': 'Resolusyon',
  'section.input': 'Input', 'section.keys': 'Mga key', 'section.apps': 'Mga app', 'section.files': 'Mga file',
  'section.sharing': 'Pagbabahagi', 'section.gamepads': 'Mga gamepad', 'section.graphs': 'Mga graph',
  'section.monitor': 'Monitor ng sistema', 'section.shortcuts': 'Mga shortcut', 'section.language': 'Wika',
  'screen.manual': 'manwal na resolusyon', 'screen.apply': 'ilapat', 'screen.scaling': 'pag-scale',
  'screen.css': 'CSS scaling (walang HiDPI)', 'audio.bitrate': 'bitrate', 'input.gaming': 'gaming mode (pointer lock)',
  'input.trackpad': 'trackpad mode', 'input.keyboard': 'keyboard sa screen', 'apps.search': 'maghanap ng app',
  'apps.install': 'i-install', 'apps.remove': 'alisin', 'apps.update': 'i-update', 'apps.run': 'patakbuhin',
  'apps.command': 'utos', 'apps.empty': 'walang nakitang app', 'apps.error': 'hindi ma-load ang listahan ng app',
  'files.open': 'buksan ang file browser', 'files.close': 'isara', 'files.upload': 'mag-upload',
  'sharing.viewOnly': 'tingin lang', 'sharing.player': 'manlalaro {n}', 'sharing.copy': 'kopyahin',
  'gamepads.touch': 'touch gamepad', 'gamepads.none': 'walang gamepad', 'monitor.memory': 'memorya',
  'shortcuts.menu': 'Menu', 'shortcuts.fullscreen': 'Buong screen', 'shortcuts.pointer': 'I-lock ang pointer',
};

const da = {
  'section.clipboard': 'Udklipsholder', 'section.stats': 'Statistik',
  'menu.title': 'Menu', 'section.video': 'Video', 'section.audio': 'Lyd', 'section.screen': 'Opløsning',
  'section.input': 'Input', 'section.keys': 'Taster', 'section.apps': 'Apps', 'section.files': 'Filer',
  'section.sharing': 'Deling', 'section.gamepads': 'Gamepads', 'section.graphs': 'Grafer',
  'section.monitor': 'Systemovervågning', 'section.shortcuts': 'Genveje', 'section.language': 'Sprog',
  'screen.manual': 'manuel opløsning', 'screen.apply': 'anvend', 'screen.scaling': 'skalering',
  'screen.css': 'CSS-skalering (ingen HiDPI)', 'audio.bitrate': 'bitrate', 'input.gaming': 'spiltilstand (låst markør)',
  'input.trackpad': 'pegefelttilstand', 'input.keyboard': 'skærmtastatur', 'apps.search': 'søg efter apps',
  'apps.install': 'installer', 'apps.remove': 'fjern', 'apps.update': 'opdater', 'apps.run': 'kør',
  'apps.command': 'kommando', 'apps.empty': 'ingen apps fundet', 'apps.error': 'app-listen kunne ikke indlæses',
  'files.open': 'åbn filbrowser', 'files.close': 'luk', 'files.upload': 'upload', 'sharing.viewOnly': 'kun visning',
  'sharing.player': 'spiller {n}', 'sharing.copy': 'kopiér', 'gamepads.touch': 'berørings-gamepad',
  'gamepads.none': 'ingen gamepads', 'monitor.memory': 'hukommelse', 'shortcuts.menu': 'Menu',
  'shortcuts.fullscreen': 'Fuld skærm', 'shortcuts.pointer': 'Lås markør',
};

export const LANGUAGES = { en, es, zh, hi, pt, fr, ru, de, tr, it, nl, ar, ko, ja, vi, th, fil, da };

// Names shown in the language picker (each in its own language).
export const LANGUAGE_NAMES = {
  en: 'English', es: 'Español', zh: '中文', hi: 'हिन्दी', pt: 'Português', fr: 'Français', ru: 'Русский',
  de: 'Deutsch', tr: 'Türkçe', it: 'Italiano', nl: 'Nederlands', ar: 'العربية', ko: '한국어', ja: '日本語',
  vi: 'Tiếng Việt', th: 'ไทย', fil: 'Filipino', da: 'Dansk',
};

const RTL = new Set(['ar']);
export const isRtl = (lang) => RTL.has(lang);

const base = (code) => String(code || '').split(/[-_]/)[0].toLowerCase();

// ?lang=xx, then the browser's languages in preference order, then English.
export function pickLanguage(search, preferred = []) {
  const m = /[?&]lang=([A-Za-z_-]+)/.exec(search || '');
  const cands = [m ? m[1] : null, ...preferred];
  for (const c of cands) {
    const b = base(c);
    if (b && b in LANGUAGES) return b;
  }
  return 'en';
}

export function interpolate(str, vars) {
  if (!vars) return str;
  return str.replace(/\{(\w+)\}/g, (all, k) => (Object.prototype.hasOwnProperty.call(vars, k) ? String(vars[k]) : all));
}

// t(key, vars): the string in `lang`, else English, else the key.
export function translator(lang) {
  const dict = LANGUAGES[base(lang)] || en;
  const t = (key, vars) => {
    const s = Object.prototype.hasOwnProperty.call(dict, key) ? dict[key] : en[key];
    return typeof s === 'string' ? interpolate(s, vars) : key;
  };
  t.lang = LANGUAGES[base(lang)] ? base(lang) : 'en';
  return t;
}
